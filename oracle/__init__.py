"""oracle — TEST INFRASTRUCTURE ONLY.

ctypes wrapper over ``libvdb_oracle.so``, the CPU restatement of the reference's
IVF-Flat CPU path (``/root/reference/engine/ivf_flat_index.cpp``, ``use_gpu=false``).
Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this package; the product (``cuda-acceleratedvectordatabaseengine_amd``)
never does.

Parity status (see DESIGN.md "Oracle"): the reference holds no golden values and
running it here was denied. The restatement is pinned by the
reference-derived known-answer test, the reference's validity rules and an
independent numpy restatement (``oracle/np_ref.py``).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "libvdb_oracle.so")
_lib = None

L2, INNER_PRODUCT, COSINE = 0, 1, 2

_f32p = ctypes.POINTER(ctypes.c_float)
_u64p = ctypes.POINTER(ctypes.c_uint64)
_u32p = ctypes.POINTER(ctypes.c_uint32)
_u8p = ctypes.POINTER(ctypes.c_uint8)


def build() -> str:
    """Compile the restatement with gcc (fp-contract off)."""
    subprocess.check_call(["make", "-s", "-C", _HERE])
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        vp = ctypes.c_void_p
        sig = {
            "oracle_create": (vp, [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int]),
            "oracle_destroy": (None, [vp]),
            "oracle_train": (None, [vp, _f32p, ctypes.c_uint64]),
            "oracle_train_seed_only": (None, [vp, _f32p, ctypes.c_uint64]),
            "oracle_add": (None, [vp, _f32p, _u64p, ctypes.c_uint64]),
            "oracle_search": (None, [vp, _f32p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, _f32p, _u64p]),
            "oracle_search_mt": (None, [vp, _f32p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, _f32p, _u64p, ctypes.c_int]),
            "oracle_search_shard": (None, [vp, _f32p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, _u8p, _f32p, _u64p]),
            "oracle_search_shard_mt": (None, [vp, _f32p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, _u8p, _f32p, _u64p, ctypes.c_int]),
            "oracle_stream_begin": (vp, [vp, _f32p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32]),
            "oracle_stream_probed": (ctypes.c_uint32, [vp, ctypes.c_uint32]),
            "oracle_stream_scan": (None, [vp, ctypes.c_uint32, ctypes.c_int]),
            "oracle_stream_finish": (None, [vp, _u8p, _f32p, _u64p]),
            "oracle_merge_ranks": (None, [_f32p, _u64p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, _f32p, _u64p]),
            "oracle_select_nprobe": (None, [vp, _f32p, ctypes.c_uint32, _u32p]),
            "oracle_assign": (None, [vp, _f32p, ctypes.c_uint64, _u32p]),
            "oracle_assign_mt": (None, [vp, _f32p, ctypes.c_uint64, _u32p, ctypes.c_int]),
            "oracle_get_centroids": (None, [vp, _f32p]),
            "oracle_set_centroids": (None, [vp, _f32p]),
            "oracle_list_count": (ctypes.c_uint64, [vp, ctypes.c_uint32]),
            "oracle_get_list": (None, [vp, ctypes.c_uint32, _f32p, _u64p]),
            "oracle_set_list": (None, [vp, ctypes.c_uint32, _f32p, _u64p, ctypes.c_uint64]),
            "oracle_total_vectors": (ctypes.c_uint64, [vp]),
            "oracle_list_set_count": (None, [vp, ctypes.c_uint32, ctypes.c_uint64]),
            "oracle_list_resize": (None, [vp, ctypes.c_uint32, ctypes.c_uint64, ctypes.POINTER(_f32p), ctypes.POINTER(_u64p)]),
            "oracle_gen_normal": (None, [ctypes.c_uint32, ctypes.c_uint64, _f32p]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def _p(a, t):
    return a.ctypes.data_as(t)


def gen_normal(seed: int, n: int) -> np.ndarray:
    """std::mt19937(seed) + std::normal_distribution<float>(0,1), n draws."""
    out = np.empty(n, dtype=np.float32)
    lib().oracle_gen_normal(seed, n, _p(out, _f32p))
    return out


def reference_test_data(n: int, q: int, d: int, seed: int = 12345):
    """Database then queries from one generator, ids 0..n-1 (gpu_vs_cpu_test.cpp:74-108)."""
    flat = gen_normal(seed, (n + q) * d)
    return flat[: n * d].reshape(n, d), flat[n * d:].reshape(q, d), np.arange(n, dtype=np.uint64)


class OracleIndex:
    """CPU restatement of IVFFlatIndex (use_gpu=false)."""

    def __init__(self, dimension: int, nlist: int, metric: int = L2):
        self.dim, self.nlist, self.metric = dimension, nlist, metric
        self._h = lib().oracle_create(dimension, nlist, metric)
        if not self._h:
            raise ValueError("Invalid configuration: dimension and nlist must be > 0")

    def __del__(self):
        h = getattr(self, "_h", None)
        if h and _lib is not None:
            _lib.oracle_destroy(h)
            self._h = None

    def train(self, vectors: np.ndarray):
        v = np.ascontiguousarray(vectors, dtype=np.float32)
        lib().oracle_train(self._h, _p(v, _f32p), v.shape[0])

    def train_seed_only(self, vectors: np.ndarray):
        v = np.ascontiguousarray(vectors, dtype=np.float32)
        lib().oracle_train_seed_only(self._h, _p(v, _f32p), v.shape[0])

    def add(self, vectors: np.ndarray, ids: np.ndarray):
        v = np.ascontiguousarray(vectors, dtype=np.float32)
        i = np.ascontiguousarray(ids, dtype=np.uint64)
        lib().oracle_add(self._h, _p(v, _f32p), _p(i, _u64p), v.shape[0])

    def search(self, queries: np.ndarray, nprobe: int, k: int, threads: int = 1):
        q = np.ascontiguousarray(queries, dtype=np.float32).reshape(-1, self.dim)
        n = q.shape[0]
        D = np.empty((n, k), dtype=np.float32)
        I = np.empty((n, k), dtype=np.uint64)
        if threads == 1:
            lib().oracle_search(self._h, _p(q, _f32p), n, nprobe, k, _p(D, _f32p), _p(I, _u64p))
        else:
            lib().oracle_search_mt(self._h, _p(q, _f32p), n, nprobe, k, _p(D, _f32p), _p(I, _u64p), threads)
        return D, I

    def search_shard(self, queries: np.ndarray, nprobe: int, k: int, owned: np.ndarray, threads: int = 1):
        q = np.ascontiguousarray(queries, dtype=np.float32).reshape(-1, self.dim)
        o = np.ascontiguousarray(owned, dtype=np.uint8)
        n = q.shape[0]
        D = np.empty((n, k), dtype=np.float32)
        I = np.empty((n, k), dtype=np.uint64)
        if threads == 1:
            lib().oracle_search_shard(self._h, _p(q, _f32p), n, nprobe, k, _p(o, _u8p), _p(D, _f32p), _p(I, _u64p))
        else:
            lib().oracle_search_shard_mt(self._h, _p(q, _f32p), n, nprobe, k, _p(o, _u8p), _p(D, _f32p),
                                         _p(I, _u64p), threads)
        return D, I

    def search_shard_streamed(self, queries: np.ndarray, nprobe: int, k: int, owned: np.ndarray, counts,
                              fill, threads: int = 0):
        """search_shard over a shard that never sits in the checker's memory whole: every
        list's count is set (emptiness), then each owned probed list is loaded alone —
        fill(l, vectors, ids) writes its rows in place — scanned for every query probing it,
        and dropped. Returns (D, I, vectors loaded)."""
        q = np.ascontiguousarray(queries, dtype=np.float32).reshape(-1, self.dim)
        o = np.ascontiguousarray(owned, dtype=np.uint8)
        n = q.shape[0]
        for l in range(self.nlist):
            self.set_list_count(l, int(counts[l]))
        st = lib().oracle_stream_begin(self._h, _p(q, _f32p), n, nprobe, k)
        loaded = 0
        try:
            for l in range(self.nlist):
                c = int(counts[l])
                if not (o[l] and c and lib().oracle_stream_probed(st, l)):
                    continue
                v, i = self.list_buffers(l, c)
                fill(l, v, i)
                lib().oracle_stream_scan(st, l, threads)
                self.set_list_count(l, c)  # (rows dropped)
                loaded += c
        finally:
            D = np.empty((n, k), dtype=np.float32)
            I = np.empty((n, k), dtype=np.uint64)
            lib().oracle_stream_finish(st, _p(o, _u8p), _p(D, _f32p), _p(I, _u64p))
        return D, I, loaded

    def select_nprobe(self, query: np.ndarray, nprobe: int) -> np.ndarray:
        q = np.ascontiguousarray(query, dtype=np.float32)
        out = np.empty(min(nprobe, self.nlist), dtype=np.uint32)
        lib().oracle_select_nprobe(self._h, _p(q, _f32p), nprobe, _p(out, _u32p))
        return out

    def assign(self, vectors: np.ndarray, threads: int = 1) -> np.ndarray:
        """assign_to_lists (cpp:259-295); threads != 1: rows over OpenMP threads (0: all),
        bit-identical per row."""
        v = np.ascontiguousarray(vectors, dtype=np.float32)
        out = np.empty(v.shape[0], dtype=np.uint32)
        if threads == 1:
            lib().oracle_assign(self._h, _p(v, _f32p), v.shape[0], _p(out, _u32p))
        else:
            lib().oracle_assign_mt(self._h, _p(v, _f32p), v.shape[0], _p(out, _u32p), threads)
        return out

    @property
    def centroids(self) -> np.ndarray:
        out = np.empty((self.nlist, self.dim), dtype=np.float32)
        lib().oracle_get_centroids(self._h, _p(out, _f32p))
        return out

    @centroids.setter
    def centroids(self, c: np.ndarray):
        c = np.ascontiguousarray(c, dtype=np.float32)
        assert c.shape == (self.nlist, self.dim)
        lib().oracle_set_centroids(self._h, _p(c, _f32p))

    def list_count(self, l: int) -> int:
        return int(lib().oracle_list_count(self._h, l))

    def get_list(self, l: int):
        n = self.list_count(l)
        v = np.empty((n, self.dim), dtype=np.float32)
        i = np.empty(n, dtype=np.uint64)
        lib().oracle_get_list(self._h, l, _p(v, _f32p), _p(i, _u64p))
        return v, i

    def set_list(self, l: int, vectors: np.ndarray, ids: np.ndarray):
        v = np.ascontiguousarray(vectors, dtype=np.float32).reshape(-1, self.dim)
        i = np.ascontiguousarray(ids, dtype=np.uint64)
        lib().oracle_set_list(self._h, l, _p(v, _f32p), _p(i, _u64p), v.shape[0])

    def set_list_count(self, l: int, count: int):
        """List l is stored on another shard: keep its count (emptiness) and no rows."""
        lib().oracle_list_set_count(self._h, l, count)

    def list_buffers(self, l: int, count: int):
        """Resize list l to `count` vectors and return writable numpy views of its
        storage (vectors (count, dim) f32, ids (count,) u64) to fill in place."""
        vp, ip = _f32p(), _u64p()
        lib().oracle_list_resize(self._h, l, count, ctypes.byref(vp), ctypes.byref(ip))
        if count == 0:
            return np.empty((0, self.dim), np.float32), np.empty(0, np.uint64)
        v = np.ctypeslib.as_array(vp, shape=(count, self.dim))
        i = np.ctypeslib.as_array(ip, shape=(count,))
        return v, i

    @property
    def total_vectors(self) -> int:
        return int(lib().oracle_total_vectors(self._h))


def merge_ranks(dist: np.ndarray, ids: np.ndarray, k: int):
    """Merge per-rank partials shaped (nranks, n, k) into (n, k)."""
    d = np.ascontiguousarray(dist, dtype=np.float32)
    i = np.ascontiguousarray(ids, dtype=np.uint64)
    r, n, _ = d.shape
    D = np.empty((n, k), dtype=np.float32)
    I = np.empty((n, k), dtype=np.uint64)
    lib().oracle_merge_ranks(_p(d, _f32p), _p(i, _u64p), r, n, k, _p(D, _f32p), _p(I, _u64p))
    return D, I
