set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/s35
timeout -k 10 1000 python -u -m pytest -q --timeout 500 --timeout-method thread -m gpu tests/ -x -p no:cacheprovider > gpurun_out/s35/full.log 2>&1
rc=$?
tail -12 gpurun_out/s35/full.log | cut -c1-300
[ $rc -ne 0 ] && exit $rc
for st in 20 50; do
timeout -k 10 200 python -u bench.py --steps $st --warmup 5 > gpurun_out/s35/b$st.log 2>&1 && python -c "import json;d=json.loads(open('gpurun_out/s35/b$st.log').read().strip().splitlines()[-1]);e=d['eigh_stats'];print($st, d['ms_per_step'], e['iters_per_gen'], e['schedule_per_gen'], e['capped'], e['max_off_rel'], d['gemm_precision'])"
done
