"""Diagnostic: check the giant list's exported contents against the source data."""
import os, sys, time
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import load_vdb
vdb = load_vdb()
n, dim, nlist = int(sys.argv[1]), 768, int(sys.argv[2])
dev = torch.device("cuda", 0)
with torch.cuda.stream(torch.cuda.Stream(dev)):
    s = torch.cuda.current_stream().cuda_stream
    data = torch.empty((n, dim), dtype=torch.float32, device=dev)
    vdb.gen_normal_device(data.data_ptr(), n * dim, seed=12345, stream=s)
    torch.cuda.synchronize()
    zr = (data.abs().sum(1) == 0)
    print("zero rows in data:", int(zr.sum()), "first", torch.nonzero(zr)[:5].flatten().tolist(), flush=True)
    nz_first = torch.nonzero(data.reshape(-1) == 0)[:5].flatten().tolist()
    print("first zero elements", nz_first, flush=True)
    ids = torch.arange(n, dtype=torch.int64, device=dev)
    idx = vdb.IVFFlatIndex(vdb.IVFFlatIndex.Config(dim, nlist))
    idx.train_device(data.data_ptr(), min(100000, n))
    idx.add_device(data.data_ptr(), ids.data_ptr(), n)
    sizes = idx.list_sizes()
    L = int(np.argmax(sizes)); c = int(sizes[L])
    print("giant list", L, c, flush=True)
    V, I = idx.get_list(L)
    print("exported ids: min", I.min(), "max", I.max(), "unique", len(np.unique(I)), flush=True)
    zrows = np.nonzero(np.abs(V).sum(1) == 0)[0]
    print("zero rows in export:", len(zrows), "first positions", zrows[:5].tolist(), "their ids", I[zrows[:5]].tolist(), flush=True)
    # compare a sample of rows against source data by id
    samp = np.linspace(0, c - 1, 2000).astype(np.int64)
    src = data[torch.from_numpy(I[samp].astype(np.int64)).to(dev)].cpu().numpy()
    bad = np.nonzero(~np.all(src == V[samp], axis=1))[0]
    print("sample rows differing from source:", len(bad), "first positions", samp[bad[:5]].tolist(), flush=True)
    # locate where corruption starts
    if len(bad):
        p = samp[bad[0]]
        print("first bad position", p, "block", p // 64, "c*dim", c * dim, "p*dim", p * dim, flush=True)
