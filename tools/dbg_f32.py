import numpy as np, torch
from nats_llm_studio_amd import ops
from nats_llm_studio_amd.gguf import quants as Q
for t in [0, 1, 30, 8, 12, 13, 14]:
    rows, K = 16, 512
    x = np.arange(rows*K, dtype=np.float32).reshape(rows, K) / 1024.0
    raw = Q.quantize(x, t)
    w = ops.QWeight(raw, t, rows, K, 'cuda')
    d = w.dense().float().cpu().numpy()
    ref = Q.dequantize(raw, t, (rows, K))
    bad = np.abs(d - ref) > 1e-2 * (np.abs(ref) + 1e-3)
    print(t, 'bad frac', bad.mean())
    if bad.any() and t == 0:
        r, k = np.argwhere(bad)[0]
        print('first bad', r, k, d[r, k], ref[r, k], 'd row0 first 70:', (d[0, :70]*1024).round(1))
        print('k where row0 bad', np.where(bad[0])[0][:40])
