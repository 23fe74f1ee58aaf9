# Ant rollout: layer 2 split over MFMA + VALU (EVOXMI_ANT_L2_MFMA = 0 / 16 / 32), A/B on one box
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_determinism_gpu.py tests/test_neuroevolution.py -m gpu -x -q --timeout 120 --timeout-method thread -k "ant or Ant" > gpurun_out/r3as_ant_tests.log 2>&1 || { tail -40 gpurun_out/r3as_ant_tests.log; exit 1; }
tail -2 gpurun_out/r3as_ant_tests.log
timeout -k 10 60 tools/k15_mfma_probe 64 > gpurun_out/r3as_k15_probe.log 2>&1 || exit 1
for km in 0 16 32 0 16; do
  EVOXMI_ANT_L2_MFMA=$km timeout -k 10 200 python -u tools/neuro_latency.py 64 8192 > gpurun_out/r3as_lat_km$km.log 2>&1 || exit 1
  echo "km=$km"; grep " 1000 " gpurun_out/r3as_lat_km$km.log
done
for km in 0 16; do
  EVOXMI_ANT_L2_MFMA=$km timeout -k 10 200 python -u tools/bench_neuro.py --pop 1024 --gens 5 --graph > gpurun_out/r3as_pop1024_km$km.log 2>&1 || exit 1
  echo "km=$km"; tail -1 gpurun_out/r3as_pop1024_km$km.log
  EVOXMI_ANT_L2_MFMA=$km timeout -k 10 300 python -u tools/bench_neuro.py --pop 8192 --gens 5 --graph > gpurun_out/r3as_pop8192_km$km.log 2>&1 || exit 1
  echo "km=$km"; tail -1 gpurun_out/r3as_pop8192_km$km.log
done
