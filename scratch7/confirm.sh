set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/s31
timeout -k 10 200 python -u tools/bench_gemm_blk.py --shapes 10000x1000x1000 > gpurun_out/s31/gemm.jsonl 2>&1 && python -c "
import json
d=[json.loads(l) for l in open('gpurun_out/s31/gemm.jsonl') if l.startswith('{')][-1]
print('h3_gemm_us', d['h3_gemm_us'])"
for st in 20 50; do
timeout -k 10 200 python -u bench.py --steps $st --warmup 5 > gpurun_out/s31/b$st.log 2>&1 && python -c "import json;d=json.loads(open('gpurun_out/s31/b$st.log').read().strip().splitlines()[-1]);e=d['eigh_stats'];print($st, d['ms_per_step'], e['iters_per_gen'], e['schedule_per_gen'], e['capped'], e['max_off_rel'])"
done
