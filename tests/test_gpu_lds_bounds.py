"""GPU parity at the boundaries of the kernels' fixed-size LDS arrays (after the
round-5 fault: the int8 calibration batch reached the plan kernel with more pairs than its
LDS arrays hold). Every kernel whose LDS is sized by batch, pairs, k or item width now has a
host-side guard (a std::length_error before the launch) and a device-side early-out; these
tests run each one AT its boundary and one step past it, where the engine must cut or split
the work, and compare ids and distance bits with the oracle (search_list_cpu /
select_nprobe_lists, ivf_flat_index.cpp:298-384):

* ivf_plan_probes sorts a batch's (query, probe) pairs in LDS arrays of kPlanMaxPairs = 8192:
  64 queries x nprobe 128 fill them exactly; nprobe 129 cuts the batch to 63 queries
  (batch_cap), for the screened scan (k 10) and the exact one (k 100);
* ivf_select_rerank keeps 4 R x 64 partial top-P entries (R = 16 at nprobe 1024, the cap) and
  stages candidate centroid rows in chunks of at most 64 (s_ci): nprobe 1024 at dim 64 makes
  more than 1024 candidates, i.e. 16+ full chunks;
* ivf_screen_collect holds 16 queries per narrow/16-wide item and 32 per 32-query item (s_thr,
  s_pst, s_qsc): a hub list probed by exactly 16 / 17 / 32 / 33 queries of a batch.
"""
import numpy as np
import pytest

import oracle
from conftest import load_vdb
from test_gpu_bounded import assert_same, hub_data, lists_pair, search_all
from test_gpu_parity import mirror_from_oracle

vdb = load_vdb()
pytestmark = pytest.mark.gpu


def _index(seed, n, dim, nlist, metric=0):
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((n, dim)).astype(np.float32)
    Q = rng.standard_normal((130, dim)).astype(np.float32)
    ids = np.arange(n, dtype=np.uint64)
    o = oracle.OracleIndex(dim, nlist, metric)
    o.centroids = X[:nlist] * 0.5
    o.add(X, ids)
    g = mirror_from_oracle(o, dim, nlist, metric)
    g.add(X, ids)
    return g, o, Q


@pytest.mark.parametrize("k", [10, 100])
def test_plan_at_its_pair_capacity(k):
    g, o, Q = _index(11 + k, 20000, 64, 160)
    g.set_batch(64)
    for nprobe in (128, 129):  # 64 x 128 = kPlanMaxPairs exactly; 129: batches of 63
        assert_same(*g.search(Q, nprobe=nprobe, k=k), *o.search(Q, nprobe, k))


@pytest.mark.parametrize("metric", [0, 1])
def test_select_rerank_at_nprobe_cap(metric):
    # nprobe 1024: R = 16 registers of partial top-P lists (s_top_*), and > 1024 candidate
    # lists re-ranked in LDS chunks of 64 rows at dim 64
    g, o, Q = _index(21 + metric, 30000, 64, 1100, metric)
    Q = Q[:40]
    for nprobe in (1023, 1024):  # (1024: the engine's nprobe cap; above it the call is refused)
        assert_same(*g.search(Q, nprobe=nprobe, k=10), *o.search(Q, nprobe, 10))


@pytest.mark.parametrize("metric", [0, 1])
def test_collect_items_at_their_width(metric):
    # every query of the batch probes the hub list: a batch of 16 / 32 queries makes one
    # item of exactly the width, 17 / 33 one item of the width plus the rest
    X, ids, lists, C, Q = hub_data(64, seed=40 + metric)
    g, o = lists_pair(X, ids, lists, C, metric)
    nprobe = 3 if metric == 0 else 6
    Dr, Ir = o.search(Q, nprobe, 10)
    for group, batches in ((16, (16, 17)), (32, (32, 33))):
        g.set_option("screen_group", group)
        for b in batches:
            assert_same(*search_all(g, Q, nprobe, 10, b), Dr, Ir)
