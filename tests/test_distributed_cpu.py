"""World-size-2 gloo test of the list-sharded search protocol on CPU.

Every rank holds the same index, owns the lists vdb_shard_plan gives it (the same
host-side LPT plan the GPU path uses), computes its partial top-k with the oracle's
per-rank semantics (stale slots included), all-gathers the partials over gloo and
merges them; the result must equal the unsharded search. The GPU path runs the
same protocol with RCCL and vdb_merge_ranks_packed_device (bench.py)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, out):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    sys.path.insert(0, os.path.join(root, "tests"))
    import oracle
    from conftest import load_vdb
    vdb = load_vdb()
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    X, Q, ids = oracle.reference_test_data(8000, 48, 16, seed=77)
    o = oracle.OracleIndex(16, 40, 0)
    o.train(X[:4000])
    o.add(X, ids)
    sizes = np.array([o.list_count(l) for l in range(40)], np.uint64)
    owner = vdb.shard_plan(sizes, world)
    D, I = o.search_shard(Q, 9, 10, (owner == rank).astype(np.uint8))
    # the packed per-rank record of vdb_rank_record_bytes: f32 dist | pad to 8 | u64 ids,
    # exchanged by ONE all-gather per batch, exactly as bench.py does over RCCL
    rec, off = vdb.rank_record_bytes(48, 10), vdb.rank_record_ids_offset(48, 10)
    mine = np.zeros(rec, np.uint8)
    mine[:D.nbytes] = D.view(np.uint8).ravel()
    mine[off:off + I.nbytes] = I.view(np.uint8).ravel()
    gathered = torch.empty(world * rec, dtype=torch.uint8)
    dist.all_gather_into_tensor(gathered, torch.from_numpy(mine))
    recs = gathered.numpy().reshape(world, rec)
    Dg = np.stack([r[:D.nbytes].view(np.float32).reshape(48, 10) for r in recs])
    Ig = np.stack([r[off:off + I.nbytes].view(np.uint64).reshape(48, 10) for r in recs])
    Dm, Im = oracle.merge_ranks(Dg, Ig, 10)
    Dr, Ir = o.search(Q, 9, 10)
    out[rank] = int(np.array_equal(Im, Ir) and np.array_equal(Dm.view(np.uint32), Dr.view(np.uint32)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_sharded_search_equals_single(world):
    ctx = mp.get_context("spawn")
    out = ctx.Array("i", [0] * world)
    mp.start_processes(_worker, args=(world, _free_port(), out), nprocs=world, start_method="spawn", join=True)
    assert list(out) == [1] * world
