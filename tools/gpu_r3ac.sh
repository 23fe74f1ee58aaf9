# flagship bench: default, with an async EvalMonitor in the timed loop, and composition / hybrid functions at d=1000
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 300 python -u bench.py > gpurun_out/r3ac_bench.log 2>&1 || exit 1
tail -1 gpurun_out/r3ac_bench.log | cut -c1-400
timeout -k 10 300 python -u bench.py --monitor > gpurun_out/r3ac_bench_monitor.log 2>&1 || exit 1
tail -1 gpurun_out/r3ac_bench_monitor.log | cut -c1-300
for f in 6 9 10 11 12; do
  timeout -k 10 300 python -u bench.py --func $f --steps 30 > gpurun_out/r3ac_bench_f$f.log 2>&1 || exit 1
  tail -1 gpurun_out/r3ac_bench_f$f.log | cut -c1-330
done
