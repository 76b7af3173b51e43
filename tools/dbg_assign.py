import sys, os, numpy as np
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo")); sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "tests"))
import torch
from conftest import golden
from pq_huffman_amd import codec
ctx = codec.Context(0)
for name in ["sift_n1000_m8_k256", "deep_n500_m16_k256"]:
    g = golden(f"pq_{name}.npz")
    x, c, want = g["x"], g["centroids"], g["codes"]
    pq = codec.PQ(ctx, c)
    got = pq.assign(torch.from_numpy(x).cuda()).cpu().numpy()
    bad = np.argwhere(got != want)
    print(name, "mismatch", len(bad), "rerank", pq.rerank_count())
    m = c.shape[0]; ds = c.shape[2]
    for v, i in bad[:10]:
        xs = x[v, i*ds:(i+1)*ds].astype(np.float64)
        d = ((xs[None, :] - c[i].astype(np.float64))**2).sum(1)
        o = np.argsort(d)
        print(f" v={v} part={i} got={got[v,i]} want={want[v,i]} d_got={d[got[v,i]]:.6g} d_want={d[want[v,i]]:.6g} best3={o[:3]} {d[o[:3]]}")
