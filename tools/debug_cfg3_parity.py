"""Diagnostic (not collected by pytest): rebuild the bench index and diff the GPU
engine against the oracle on a few queries, printing the first mismatches."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle  # noqa: E402
from conftest import load_vdb  # noqa: E402

vdb = load_vdb()


def main():
    n, dim, nlist, nprobe, k = int(sys.argv[1]), 768, int(sys.argv[2]), 32, 10
    dev = torch.device("cuda", 0)
    with torch.cuda.stream(torch.cuda.Stream(dev)):
        s = torch.cuda.current_stream().cuda_stream
        data = torch.empty((n, dim), dtype=torch.float32, device=dev)
        vdb.gen_normal_device(data.data_ptr(), n * dim, seed=12345, stream=s)
        ids = torch.arange(n, dtype=torch.int64, device=dev)
        q = torch.empty((8, dim), dtype=torch.float32, device=dev)
        vdb.gen_normal_device(q.data_ptr(), 8 * dim, seed=12346, stream=s)
        torch.cuda.synchronize()
        idx = vdb.IVFFlatIndex(vdb.IVFFlatIndex.Config(dim, nlist))
        t = time.time()
        idx.train_device(data.data_ptr(), min(100000, n))
        idx.add_device(data.data_ptr(), ids.data_ptr(), n)
        print("build", time.time() - t, flush=True)
        sizes = idx.list_sizes()
        print("sizes max", sizes.max(), "top", np.sort(sizes)[-8:], "empty", (sizes == 0).sum(), flush=True)
        Q = q.cpu().numpy()
        o = oracle.OracleIndex(dim, nlist, 0)
        o.centroids = idx.centroids
        for l in range(nlist):          # full mirror
            v, i = o.list_buffers(l, int(sizes[l]))
            if len(i):
                idx.get_list_into(l, v, i)
        # host-side sanity: a few lists from the device agree with a direct recompute of membership
        A = o.assign(data[:20000].cpu().numpy())
        print("assign check", np.array_equal(np.sort(A), np.sort(A)), flush=True)
        for call in (1, 4):
            for c0 in range(0, 8, call):
                Qc = Q[c0:c0 + call]
                Dg, Ig = idx.search(Qc, nprobe=nprobe, k=k)
                Do, Io = o.search(Qc, nprobe, k)
                same_i = np.array_equal(Ig, Io)
                same_d = np.array_equal(Dg.view(np.uint32), Do.view(np.uint32))
                print(f"call={call} q0={c0} ids_equal={same_i} dist_bits_equal={same_d}", flush=True)
                if not (same_i and same_d):
                    for r in range(Qc.shape[0]):
                        print("  gpu ", Ig[r].tolist(), Dg[r].tolist())
                        print("  orac", Io[r].tolist(), Do[r].tolist())
                    pg = o.select_nprobe(Qc[0], nprobe)
                    print("  probes", pg.tolist(), "sizes", sizes[pg].tolist())
                    return


if __name__ == "__main__":
    main()
