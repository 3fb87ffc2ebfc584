"""Diagnostic: build the bench index and dump centroids, list sizes and queries (npz)."""
import os, sys
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
    ids = torch.arange(n, dtype=torch.int64, device=dev)
    q = torch.empty((1280, dim), dtype=torch.float32, device=dev)
    vdb.gen_normal_device(q.data_ptr(), 1280 * dim, seed=12346, stream=s)
    torch.cuda.synchronize()
    idx = vdb.IVFFlatIndex(vdb.IVFFlatIndex.Config(dim, nlist))
    idx.train_device(data.data_ptr(), min(100000, n))
    idx.add_device(data.data_ptr(), ids.data_ptr(), n)
    np.savez_compressed(os.path.join(ROOT, "gpurun_out", f"index_{n}_{nlist}.npz"), centroids=idx.centroids,
                        sizes=idx.list_sizes(), queries=q.cpu().numpy())
    print("ok", idx.list_sizes().max())
