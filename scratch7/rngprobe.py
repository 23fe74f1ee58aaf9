import json, time, torch
from evoxmi import random as rnd
from evoxmi.ops import linalg
key = rnd.PRNGKey(99)
zc = rnd.normal(key, (1 << 22,))
zg = rnd.normal(key.cuda(), (1 << 22,)).cpu()
err = (zc - zg).abs()
kg = key.cuda()
out = linalg.normal_h3_planes(kg, 10000, 1000)
for _ in range(5):
    linalg.normal_h3_planes(kg, 10000, 1000, out=out)
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(200):
    linalg.normal_h3_planes(kg, 10000, 1000, out=out)
torch.cuda.synchronize()
us = (time.perf_counter() - t) / 200 * 1e6
print(json.dumps({"max_abs_err_vs_host": float(err.max()), "max_rel_err_abs_gt_0.1": float((err / zc.abs())[zc.abs() > 0.1].max()),
                  "mean_g": float(zg.mean()), "std_g": float(zg.std()), "philox_h_10000x1000_us": round(us, 2)}))
