set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/split
for r in 4 8 4 8; do
  EVOXMI_SPLIT_ROWS=$r timeout -k 10 120 python -u tools/bench_gemm_blk.py --only-split --reps 50 --shapes 10000x1000x1000,5000x1000x1000,1250x1000x1000 >> gpurun_out/split/sweep.jsonl 2>gpurun_out/split/err.log || { tail -5 gpurun_out/split/err.log; exit 1; }
done
cat gpurun_out/split/sweep.jsonl
for r in 4 8; do
  EVOXMI_SPLIT_ROWS=$r timeout -k 10 200 python -u bench.py --steps 50 --warmup 5 --phase-steps 0 > gpurun_out/split/b50_$r.log 2>&1 || { tail -5 gpurun_out/split/b50_$r.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/split/b50_$r.log').read().strip().splitlines()[-1]);print('rows', $r, d['ms_per_step'], d['eigh_stats']['capped'])"
done
EVOXMI_SPLIT_ROWS=8 timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -x -p no:cacheprovider tests/test_gemm_blk.py tests/test_kernels_gpu.py -k "h3 or blk or cec2022" > gpurun_out/split/t.log 2>&1; rc=$?; tail -2 gpurun_out/split/t.log; exit $rc
