set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/s1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s1/smoke.log 2>&1 || { tail -20 gpurun_out/s1/smoke.log; exit 1; }
tail -1 gpurun_out/s1/smoke.log
for st in 20 50; do
timeout -k 10 200 python -u bench.py --steps $st --warmup 5 > gpurun_out/s1/b$st.log 2>&1 && python -c "import json;d=json.loads(open('gpurun_out/s1/b$st.log').read().strip().splitlines()[-1]);e=d['eigh_stats'];print($st, d['ms_per_step'], e['iters_per_gen'], e['schedule_per_gen'], e['capped'], e['max_off_rel'], d['phases_ms_eager'])" || exit 1
done
