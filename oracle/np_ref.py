"""oracle/np_ref.py — TEST INFRASTRUCTURE ONLY.

An independent numpy restatement of the reference's IVF-Flat CPU search path
(/root/reference/engine/ivf_flat_index.cpp, use_gpu=false), used to cross-check
the C++ restatement in oracle/cpu_ref.cpp on small cases. numpy float32 ufuncs
round every op separately (no FMA), and the loops below keep the reference's
d = 0..D-1 summation order, so distances are bit-identical to the C++ path.
"""
from __future__ import annotations

import numpy as np

L2, INNER_PRODUCT, COSINE = 0, 1, 2
U64MAX = np.uint64(0xFFFFFFFFFFFFFFFF)
FLTMAX = np.float32(np.finfo(np.float32).max)


def distances(metric: int, Q: np.ndarray, X: np.ndarray) -> np.ndarray:
    """(nq, n) fp32 distances, summed in d order (cpp:308-318, 352-362)."""
    Q = np.asarray(Q, np.float32)
    X = np.asarray(X, np.float32)
    acc = np.zeros((Q.shape[0], X.shape[0]), np.float32)
    if metric == COSINE:          # no CPU branch: distance stays 0 (cpp:351-362)
        return acc
    for d in range(Q.shape[1]):
        if metric == L2:
            diff = Q[:, d:d + 1] - X[None, :, d]
            acc = acc + diff * diff
        else:
            acc = acc + Q[:, d:d + 1] * X[None, :, d]
    return acc if metric == L2 else -acc


def select_nprobe(metric, centroids, q, nprobe):
    """select_nprobe_lists (cpp:298-336): ascending (dist, list_id)."""
    cd = distances(metric, q[None, :], centroids)[0]
    order = np.lexsort((np.arange(len(cd)), cd))
    return order[: min(nprobe, len(cd))]


def assign(metric, centroids, X):
    """assign_to_lists (cpp:259-295): first index of the minimum (strict '<')."""
    out = np.empty(X.shape[0], np.uint32)
    for i in range(0, X.shape[0], 4096):
        D = distances(metric, X[i:i + 4096], centroids)
        out[i:i + 4096] = np.argmin(D, axis=1)   # argmin returns the first minimum
    return out


def _topk(dist, ids, k):
    order = np.lexsort((ids, dist))[:k]
    return list(zip(dist[order].tolist(), ids[order].tolist()))


def _merge(slots, k):
    """merge_results (cpp:474-518)."""
    cands = sorted(c for s in slots for c in s if c[1] != int(U64MAX))
    seen, uniq = set(), []
    for c in cands:
        if c[1] not in seen:
            seen.add(c[1])
            uniq.append(c)
    D = np.full(k, FLTMAX, np.float32)
    I = np.full(k, U64MAX, np.uint64)
    for j, (d, i) in enumerate(uniq[:k]):
        D[j], I[j] = d, i
    return D, I


def search(metric, centroids, lists, queries, nprobe, k):
    """IVFFlatIndex::search (cpp:205-256). lists: [(vectors (n,D) f32, ids (n,) u64)].

    Slots persist across queries of one call (cpp:210-211), so an empty probed list
    leaves the previous query's slot content in place."""
    nlist = centroids.shape[0]
    P = min(nprobe, nlist)
    slots = [[] for _ in range(P)]
    Dout = np.empty((queries.shape[0], k), np.float32)
    Iout = np.empty((queries.shape[0], k), np.uint64)
    for qi, q in enumerate(np.asarray(queries, np.float32)):
        for p, l in enumerate(select_nprobe(metric, centroids, q, nprobe)):
            vecs, ids = lists[l]
            if len(ids) == 0:
                continue
            d = distances(metric, q[None, :], vecs)[0]
            slots[p] = _topk(d, np.asarray(ids, np.uint64), min(k, len(ids)))
        Dout[qi], Iout[qi] = _merge(slots, k)
    return Dout, Iout


def lloyd(metric, X, centroids, iters=10):
    """The Lloyd refinement of train (cpp:107-142) from given seeds; sums run in
    vector order per cluster, one float32 row add at a time."""
    C = np.array(centroids, np.float32, copy=True)
    X = np.asarray(X, np.float32)
    for _ in range(iters):
        a = assign(metric, C, X)
        sums = np.zeros_like(C)
        counts = np.zeros(C.shape[0], np.uint32)
        for i in range(X.shape[0]):
            sums[a[i]] = sums[a[i]] + X[i]
            counts[a[i]] += 1
        nz = counts > 0
        C[nz] = sums[nz] / counts[nz, None].astype(np.float32)
    return C
