set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/s15
PYTHONPATH=. timeout -k 10 120 python -u scratch7/rngprobe.py > gpurun_out/s15/rng.json 2>&1 || { tail gpurun_out/s15/rng.json; exit 1; }
cat gpurun_out/s15/rng.json | tail -1
timeout -k 10 900 python -u -m pytest -q --timeout 400 --timeout-method thread -m gpu tests/ -x -p no:cacheprovider > gpurun_out/s15/full.log 2>&1
rc=$?
tail -15 gpurun_out/s15/full.log | cut -c1-300
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/s15/b20.log 2>&1 && tail -1 gpurun_out/s15/b20.log | cut -c1-300
timeout -k 10 200 python -u bench.py --steps 50 --warmup 5 > gpurun_out/s15/b50.log 2>&1 && tail -1 gpurun_out/s15/b50.log | cut -c1-300
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/s15/kt -o kt --output-format csv -- python3 $R/bench.py --steps 40 --warmup 5 --phase-steps 0 > $R/gpurun_out/s15/kt_bench.log 2>&1 || { cd $R; tail -20 gpurun_out/s15/kt_bench.log; exit 1; }
cd $R
f=$(find gpurun_out/s15/kt -name '*kernel_trace.csv' | head -1)
python tools/ktrace_gen.py $f --marker philox_h --show -2 --agg 20 > gpurun_out/s15/kt_gen.txt
grep "philox_h\|us/gen total\|wall" gpurun_out/s15/kt_gen.txt | cut -c1-160 | tail -8
rm -f $f
