set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/s19
timeout -k 10 200 python -u tools/bench_gemm_blk.py --shapes 10000x1000x1000 > gpurun_out/s19/w8.jsonl 2>&1 || { tail gpurun_out/s19/w8.jsonl; exit 1; }
EVOXMI_H3_WAVES=4 timeout -k 10 200 python -u tools/bench_gemm_blk.py --shapes 10000x1000x1000 > gpurun_out/s19/w4.jsonl 2>&1 || { tail gpurun_out/s19/w4.jsonl; exit 1; }
python - <<'PY'
import json
for f in ("w8", "w4"):
    d = [json.loads(l) for l in open(f"gpurun_out/s19/{f}.jsonl") if l.startswith("{")][-1]
    print(f, d.get("h3_gemm_us"), d.get("h3_pct_x3_ceiling"))
PY
EVOXMI_H3_WAVES=4 timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gemm_blk.py tests/test_cec_device.py -x -p no:cacheprovider > gpurun_out/s19/t.log 2>&1 || { tail -30 gpurun_out/s19/t.log | cut -c1-300; exit 1; }
tail -1 gpurun_out/s19/t.log
EVOXMI_H3_WAVES=4 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/s19/b20w4.log 2>&1 && tail -1 gpurun_out/s19/b20w4.log | cut -c1-250
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/s19/b20w8.log 2>&1 && tail -1 gpurun_out/s19/b20w8.log | cut -c1-250
