set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/s9
timeout -k 10 300 python tools/xnorm_probe.py --gens 30 --solves 2 > gpurun_out/s9/xnorm.jsonl 2>gpurun_out/s9/err || { tail gpurun_out/s9/err; exit 1; }
cat gpurun_out/s9/xnorm.jsonl | cut -c1-300
timeout -k 10 200 python tools/bench_gemm_x3.py --reps 100 > gpurun_out/s9/gemm.jsonl 2>>gpurun_out/s9/err || { tail gpurun_out/s9/err; exit 1; }
grep "column" gpurun_out/s9/gemm.jsonl
for p in x6 x3; do
EVOXMI_SBR_CORR_PREC=$p timeout -k 10 600 python -u -m pytest -x -q --timeout 500 --timeout-method thread -m gpu tests/test_eigh_sbr.py -k "trajectory or library" > gpurun_out/s9/parity_$p.log 2>&1; echo "parity $p rc=$?"; grep -o "AssertionError.*" gpurun_out/s9/parity_$p.log | head -2; tail -1 gpurun_out/s9/parity_$p.log
done
