# round-3 end check: full GPU suite, smoke, bench (20 / 50 steps), kernel stats of the bench
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/final_gpu_tests.log 2>&1 || { tail -40 gpurun_out/final_gpu_tests.log; exit 1; }
tail -2 gpurun_out/final_gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1 || { tail -30 gpurun_out/final_smoke.log; exit 1; }
tail -2 gpurun_out/final_smoke.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/final_bench20.log 2>&1 || { tail -30 gpurun_out/final_bench20.log; exit 1; }
tail -1 gpurun_out/final_bench20.log
timeout -k 10 300 python bench.py --steps 50 --warmup 3 > gpurun_out/final_bench50.log 2>&1 || { tail -30 gpurun_out/final_bench50.log; exit 1; }
tail -1 gpurun_out/final_bench50.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/final_prof -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 3 > $R/gpurun_out/final_prof.log 2>&1 || { tail -20 $R/gpurun_out/final_prof.log; exit 1; }
cd $R && python tools/kstats.py $(find gpurun_out/final_prof -name '*kernel_stats.csv' | head -1) 23 30 > gpurun_out/final_kstats.txt 2>&1; head -30 gpurun_out/final_kstats.txt
T=$(find gpurun_out/final_prof -name '*kernel_trace.csv' | head -1)
python tools/ktrace_gen.py "$T" > gpurun_out/final_gen_timeline.txt 2>&1 || true
grep "^gen" gpurun_out/final_gen_timeline.txt | tail -8
python - "$T" > gpurun_out/final_copy_launches.txt 2>&1 <<'PY' || true
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
names = [r["Kernel_Name"] for r in rows]
gens = sum("philox_fill" in n for n in names)
cp = sum(("copyBuffer" in n) or ("elementwise_kernel" in n and "copy" in n) or ("multi_tensor" in n) for n in names)
print(f"kernels {len(names)}  marker generations {gens}  copy-like launches {cp}  per generation {cp / max(gens, 1):.2f}")
PY
cat gpurun_out/final_copy_launches.txt
