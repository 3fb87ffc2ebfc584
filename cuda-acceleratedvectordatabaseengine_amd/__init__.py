"""MI355X-native IVF-Flat search engine — Python host mirror of the reference API.

The product is ``lib/libvdb_ivf.so`` (hand-written gfx950 HIP kernels behind the C ABI
in ``include/vdb_ivf.h``). This module binds that ABI with ctypes and mirrors the
reference's ``vdb::IVFFlatIndex`` surface (``engine/ivf_flat_index.h:14-67``):
``Config``, ``SearchParams``, ``train``, ``add``, ``search``, ``warmup_lists``,
``evict_list``, ``get_gpu_memory_usage``, ``get_total_vectors``, plus the
device-resident and list-sharded forms used by ``bench.py``.

There is no CPU fallback: if the library is missing or no GPU is present, calls
raise. Import under any name, e.g. ``importlib`` with the directory path
(the directory name is not a Python identifier); ``load()`` below does that.
"""
from __future__ import annotations

import ctypes
import enum
import os
import subprocess
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("VDB_IVF_LIB") or os.path.join(_HERE, "lib", "libvdb_ivf.so")  # override: A/B builds
CPP_LIB_PATH = os.path.join(_HERE, "lib", "libvdb_ivf_cpp.so")
HEADER = os.path.join(os.path.dirname(_HERE), "include", "vdb_ivf.h")

_lib = None


class Metric(enum.IntEnum):
    """kernels::Metric (engine/kernels.cuh:24-28)."""
    L2 = 0
    InnerProduct = 1
    Cosine = 2


class VdbError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"vdb error {code}: {msg}")
        self.code = code


class _Config(ctypes.Structure):
    _fields_ = [("dimension", ctypes.c_uint32), ("nlist", ctypes.c_uint32), ("metric", ctypes.c_int32),
                ("use_gpu", ctypes.c_int32), ("max_gpu_memory", ctypes.c_uint64), ("device", ctypes.c_int32)]


class CacheStats(ctypes.Structure):
    _fields_ = [("capacity_bytes", ctypes.c_uint64), ("resident_bytes", ctypes.c_uint64),
                ("resident_lists", ctypes.c_uint64), ("loads", ctypes.c_uint64), ("evictions", ctypes.c_uint64),
                ("bytes_loaded", ctypes.c_uint64), ("file_bytes_read", ctypes.c_uint64),
                ("subbatches", ctypes.c_uint64), ("prefetches", ctypes.c_uint64), ("sync_loads", ctypes.c_uint64),
                ("io_uring", ctypes.c_int32), ("o_direct", ctypes.c_int32),
                ("screen_resident", ctypes.c_int32), ("reserved", ctypes.c_int32), ("screen_bytes", ctypes.c_uint64),
                ("screen_batches", ctypes.c_uint64), ("screen_rows_fetched", ctypes.c_uint64),
                ("screen_row_bytes", ctypes.c_uint64), ("screen_reruns", ctypes.c_uint64),
                ("screen_rows_cached", ctypes.c_uint64), ("screen_fallbacks", ctypes.c_uint64)]

    def as_dict(self):
        return {f: getattr(self, f) for f, _ in self._fields_}


class Profile(ctypes.Structure):
    _fields_ = [("batches", ctypes.c_uint64), ("scan_launches", ctypes.c_uint64), ("scan_ms", ctypes.c_double),
                ("coarse_ms", ctypes.c_double), ("total_ms", ctypes.c_double), ("scan_vectors", ctypes.c_uint64),
                ("distinct_lists", ctypes.c_uint64), ("work_items", ctypes.c_uint64),
                ("scan_bytes", ctypes.c_uint64), ("pair_vectors", ctypes.c_uint64),
                ("exact_reranks", ctypes.c_uint64), ("bounded_blocks", ctypes.c_uint64),
                ("computed_vectors", ctypes.c_uint64), ("local_merge_ms", ctypes.c_double),
                ("exchanges", ctypes.c_uint64), ("exchange_ms", ctypes.c_double), ("rank_merge_ms", ctypes.c_double),
                ("screen_collected", ctypes.c_uint64), ("collect_ms", ctypes.c_double),
                ("recheck_ms", ctypes.c_double), ("screen_floor_batches", ctypes.c_uint64),
                ("screen_floor_trips", ctypes.c_uint64), ("screen_shadow", ctypes.c_uint32),
                ("reserved0", ctypes.c_uint32)]

    def as_dict(self):
        return {f: getattr(self, f) for f, _ in self._fields_}


def build(jobs: int = 8) -> str:
    """Compile the HIP library for gfx950 (hipcc; cross-compiles without a GPU)."""
    subprocess.check_call(["make", "-s", f"-j{jobs}", "-C", _HERE])
    return LIB_PATH


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is missing: build it with `make -C {_HERE}` (no CPU fallback exists)")
    # torch ships its own libamdhip64 (SONAME libamdhip64.so.7). Loading torch first
    # lets libvdb_ivf.so bind to that same HIP runtime by SONAME, so torch tensors and
    # streams and this library share one runtime; the other order loads two.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = ctypes.CDLL(LIB_PATH)
    vp, u32, u64, i32 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int32
    sigs = {
        "vdb_last_error": (ctypes.c_char_p, []),
        "vdb_version": (ctypes.c_char_p, []),
        "vdb_build_id": (ctypes.c_char_p, []),
        "vdb_device_count": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int)]),
        "vdb_ivf_create": (ctypes.c_int, [ctypes.POINTER(_Config), ctypes.POINTER(vp)]),
        "vdb_ivf_destroy": (ctypes.c_int, [vp]),
        "vdb_ivf_train": (ctypes.c_int, [vp, vp, u64]),
        "vdb_ivf_train_device": (ctypes.c_int, [vp, vp, u64]),
        "vdb_ivf_set_centroids": (ctypes.c_int, [vp, vp]),
        "vdb_ivf_get_centroids": (ctypes.c_int, [vp, vp]),
        "vdb_ivf_add": (ctypes.c_int, [vp, vp, vp, u64]),
        "vdb_ivf_add_device": (ctypes.c_int, [vp, vp, vp, u64]),
        "vdb_ivf_search": (ctypes.c_int, [vp, vp, u32, u32, u32, vp, vp]),
        "vdb_ivf_search_device": (ctypes.c_int, [vp, vp, u32, u32, u32, vp, vp, vp]),
        "vdb_ivf_set_shard": (ctypes.c_int, [vp, u32, u32]),
        "vdb_ivf_plan_shard": (ctypes.c_int, [vp, u32, u32, vp]),
        "vdb_ivf_assign_device": (ctypes.c_int, [vp, vp, u64, vp]),
        "vdb_ivf_add_to_lists_device": (ctypes.c_int, [vp, vp, vp, vp, u64]),
        "vdb_ivf_save": (ctypes.c_int, [vp, ctypes.c_char_p]),
        "vdb_ivf_load": (ctypes.c_int, [vp, ctypes.c_char_p]),
        "vdb_merge_ranks_device": (ctypes.c_int, [vp, vp, u32, u32, u32, vp, vp, vp]),
        "vdb_shard_plan": (ctypes.c_int, [vp, u32, u32, vp]),
        "vdb_shard_plan_probe_weighted": (ctypes.c_int, [vp, vp, u64, u32, u32, u32, vp]),
        "vdb_ivf_probe_census": (ctypes.c_int, [vp, vp, u64, u32, vp]),
        "vdb_ivf_set_shard_owners": (ctypes.c_int, [vp, u32, u32, vp]),
        "vdb_ivf_plan_shard_owners": (ctypes.c_int, [vp, u32, u32, vp, vp]),
        "vdb_rank_record_bytes": (u64, [u32, u32]),
        "vdb_merge_ranks_packed_device": (ctypes.c_int, [vp, u32, u32, u32, vp, vp, vp]),
        "vdb_ivf_warmup": (ctypes.c_int, [vp, vp, u32]),
        "vdb_ivf_evict": (ctypes.c_int, [vp, u32]),
        "vdb_ivf_gpu_bytes": (u64, [vp]),
        "vdb_ivf_gpu_bytes_allocated": (u64, [vp]),
        "vdb_ivf_ntotal": (u64, [vp]),
        "vdb_ivf_list_sizes": (ctypes.c_int, [vp, vp]),
        "vdb_ivf_get_list": (ctypes.c_int, [vp, u32, vp, vp]),
        "vdb_ivf_set_batch": (ctypes.c_int, [vp, u32]),
        "vdb_ivf_set_stale_slots": (ctypes.c_int, [vp, i32]),
        "vdb_ivf_set_coarse_mode": (ctypes.c_int, [vp, i32]),
        "vdb_ivf_set_option": (ctypes.c_int, [vp, ctypes.c_char_p, ctypes.c_int64]),
        "vdb_ivf_coalesce_stats": (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]),
        "vdb_ivf_cache_stats": (ctypes.c_int, [vp, ctypes.POINTER(CacheStats)]),
        "vdb_ivf_fill_row_cache": (ctypes.c_int, [vp, vp]),
        "vdb_ivf_survivor_histogram": (ctypes.c_int, [vp, vp]),
        "vdb_ivf_collect_stamps": (ctypes.c_int, [vp, ctypes.c_void_p, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64),
                                                  ctypes.POINTER(ctypes.c_uint64)]),
        "vdb_ivf_open_lists": (ctypes.c_int, [vp, ctypes.c_char_p]),
        "vdb_ivf_profile_enable": (ctypes.c_int, [vp, i32]),
        "vdb_ivf_profile_reset": (ctypes.c_int, [vp]),
        "vdb_ivf_profile_read": (ctypes.c_int, [vp, ctypes.POINTER(Profile)]),
        "vdb_ivf_synchronize": (ctypes.c_int, [vp]),
        "vdb_ivf_stream": (vp, [vp]),
        "vdb_gen_normal_device": (ctypes.c_int, [vp, u64, u64, u64, vp]),
        "vdb_gen_mixture_device": (ctypes.c_int, [vp, u64, u32, vp, u32, ctypes.c_float, u64, u64, vp]),
        "vdb_comm_unique_id": (ctypes.c_int, [vp]),
        "vdb_ivf_attach_comm": (ctypes.c_int, [vp, vp, u32, u32]),
        "vdb_ivf_detach_comm": (ctypes.c_int, [vp]),
        "vdb_ivf_comm_status": (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]),
        "vdb_ivf_create_group": (ctypes.c_int, [ctypes.POINTER(_Config), vp, u32, ctypes.POINTER(vp)]),
        "vdb_ivf_group_size": (u32, [vp]),
        "vdb_ivf_list_owners": (ctypes.c_int, [vp, vp]),
    }
    for name, (res, args) in sigs.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def _check(rc: int):
    if rc != 0:
        raise VdbError(rc, lib().vdb_last_error().decode())


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def build_id() -> str:
    """Hash of the sources behind the scan kernels of the loaded library (vdb_build_id)."""
    return lib().vdb_build_id().decode()


def device_count() -> int:
    c = ctypes.c_int(0)
    _check(lib().vdb_device_count(ctypes.byref(c)))
    return c.value


def shard_plan(list_sizes, world: int) -> np.ndarray:
    """LPT owner rank of every list (host-only, identical on every rank)."""
    s = np.ascontiguousarray(list_sizes, dtype=np.uint64)
    out = np.empty(len(s), dtype=np.uint32)
    _check(lib().vdb_shard_plan(_ptr(s), len(s), world, _ptr(out)))
    return out


def shard_plan_probe_weighted(list_sizes, probe_counts, n_sample: int, batch: int, world: int) -> np.ndarray:
    """LPT owner of every list over the expected scan cost per batch (probe census weights)."""
    s = np.ascontiguousarray(list_sizes, dtype=np.uint64)
    c = np.ascontiguousarray(probe_counts, dtype=np.uint64)
    out = np.empty(len(s), dtype=np.uint32)
    _check(lib().vdb_shard_plan_probe_weighted(_ptr(s), _ptr(c), n_sample, batch, len(s), world, _ptr(out)))
    return out


def gen_normal_device(ptr: int, n: int, seed: int, offset: int = 0, stream: int | None = None):
    """Fill n fp32 at device address ``ptr`` with deterministic N(0,1) draws."""
    _check(lib().vdb_gen_normal_device(ctypes.c_void_p(ptr), n, seed, offset, ctypes.c_void_p(stream or 0)))


def gen_mixture_device(ptr: int, rows: int, dim: int, centers_ptr: int, ncomp: int, sigma: float, seed: int,
                       row0: int = 0, stream: int | None = None):
    """Fill rows x dim fp32 at ``ptr`` with Gaussian-mixture draws around the ncomp x dim
    device centers (synthetic clustered data; rows row0.. of one deterministic stream)."""
    _check(lib().vdb_gen_mixture_device(ctypes.c_void_p(ptr), rows, dim, ctypes.c_void_p(centers_ptr), ncomp,
                                        ctypes.c_float(sigma), seed, row0, ctypes.c_void_p(stream or 0)))


def merge_ranks_device(dist_ptr: int, ids_ptr: int, nranks: int, n: int, k: int, out_dist_ptr: int,
                       out_ids_ptr: int, stream: int | None = None):
    _check(lib().vdb_merge_ranks_device(ctypes.c_void_p(dist_ptr), ctypes.c_void_p(ids_ptr), nranks, n, k,
                                        ctypes.c_void_p(out_dist_ptr), ctypes.c_void_p(out_ids_ptr),
                                        ctypes.c_void_p(stream or 0)))


COMM_ID_BYTES = 128  # VDB_COMM_ID_BYTES


def comm_unique_id() -> bytes:
    """A fresh RCCL communicator id (rank 0 draws it and shares it with the other ranks)."""
    buf = ctypes.create_string_buffer(COMM_ID_BYTES)
    _check(lib().vdb_comm_unique_id(buf))
    return buf.raw


def rank_record_bytes(n: int, k: int) -> int:
    """Bytes of one rank's packed partial record (f32 dist [n][k], pad to 8, u64 ids [n][k])."""
    return int(lib().vdb_rank_record_bytes(n, k))


def rank_record_ids_offset(n: int, k: int) -> int:
    return (n * k * 4 + 7) // 8 * 8


def merge_ranks_packed_device(records_ptr: int, nranks: int, n: int, k: int, out_dist_ptr: int, out_ids_ptr: int,
                              stream: int | None = None):
    _check(lib().vdb_merge_ranks_packed_device(ctypes.c_void_p(records_ptr), nranks, n, k,
                                               ctypes.c_void_p(out_dist_ptr), ctypes.c_void_p(out_ids_ptr),
                                               ctypes.c_void_p(stream or 0)))


class IVFFlatIndex:
    """vdb::IVFFlatIndex (engine/ivf_flat_index.h:14-67) on one MI355X."""

    @dataclass
    class Config:
        dimension: int
        nlist: int
        metric: Metric = Metric.L2
        use_gpu: bool = True
        max_gpu_memory: int = 8 << 30
        device: int = 0
        devices: tuple = ()  # > 1 entries: one index sharded by list over these GPUs (group handle)

    @dataclass
    class SearchParams:
        nprobe: int = 10
        k: int = 10
        use_exact_rerank: bool = False  # accepted, unused — as in the reference

    def __init__(self, config: "IVFFlatIndex.Config"):
        self.config = config
        if config.dimension <= 0 or config.nlist <= 0:
            raise ValueError("Invalid configuration: dimension and nlist must be > 0")
        c = _Config(config.dimension, config.nlist, int(config.metric), int(config.use_gpu),
                    config.max_gpu_memory, config.device)
        h = ctypes.c_void_p()
        if config.devices:
            devs = (ctypes.c_int * len(config.devices))(*config.devices)
            _check(lib().vdb_ivf_create_group(ctypes.byref(c), devs, len(config.devices), ctypes.byref(h)))
        else:
            _check(lib().vdb_ivf_create(ctypes.byref(c), ctypes.byref(h)))
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            lib().vdb_ivf_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def dimension(self) -> int:
        return self.config.dimension

    # ---- build ----
    def train(self, vectors: np.ndarray):
        v = np.ascontiguousarray(vectors, dtype=np.float32).reshape(-1, self.dimension)
        _check(lib().vdb_ivf_train(self._h, _ptr(v), v.shape[0]))

    def train_device(self, ptr: int, n: int):
        _check(lib().vdb_ivf_train_device(self._h, ctypes.c_void_p(ptr), n))

    def add(self, vectors: np.ndarray, ids: np.ndarray):
        v = np.ascontiguousarray(vectors, dtype=np.float32).reshape(-1, self.dimension)
        i = np.ascontiguousarray(ids, dtype=np.uint64)
        if i.shape[0] != v.shape[0]:
            raise ValueError("vectors and ids differ in length")
        _check(lib().vdb_ivf_add(self._h, _ptr(v), _ptr(i), v.shape[0]))

    def add_device(self, vec_ptr: int, ids_ptr: int, n: int):
        _check(lib().vdb_ivf_add_device(self._h, ctypes.c_void_p(vec_ptr), ctypes.c_void_p(ids_ptr), n))

    def assign_device(self, vec_ptr: int, n: int, lists_ptr: int):
        """Exact nearest-centroid list of n device rows into u32 lists_ptr (assign_to_lists, cpp:259-295)."""
        _check(lib().vdb_ivf_assign_device(self._h, ctypes.c_void_p(vec_ptr), n, ctypes.c_void_p(lists_ptr)))

    def add_to_lists_device(self, vec_ptr: int, ids_ptr: int, lists_ptr: int, n: int):
        _check(lib().vdb_ivf_add_to_lists_device(self._h, ctypes.c_void_p(vec_ptr), ctypes.c_void_p(ids_ptr),
                                                 ctypes.c_void_p(lists_ptr), n))

    @property
    def centroids(self) -> np.ndarray:
        out = np.empty((self.config.nlist, self.dimension), dtype=np.float32)
        _check(lib().vdb_ivf_get_centroids(self._h, _ptr(out)))
        return out

    @centroids.setter
    def centroids(self, c: np.ndarray):
        c = np.ascontiguousarray(c, dtype=np.float32).reshape(self.config.nlist, self.dimension)
        _check(lib().vdb_ivf_set_centroids(self._h, _ptr(c)))

    # ---- search ----
    def search(self, queries: np.ndarray, params: "IVFFlatIndex.SearchParams | None" = None, *,
               nprobe: int | None = None, k: int | None = None):
        p = params or IVFFlatIndex.SearchParams()
        nprobe = p.nprobe if nprobe is None else nprobe
        k = p.k if k is None else k
        q = np.ascontiguousarray(queries, dtype=np.float32).reshape(-1, self.dimension)
        n = q.shape[0]
        D = np.empty((n, k), dtype=np.float32)
        I = np.empty((n, k), dtype=np.uint64)
        _check(lib().vdb_ivf_search(self._h, _ptr(q), n, nprobe, k, _ptr(D), _ptr(I)))
        return D, I

    def search_device(self, q_ptr: int, n: int, nprobe: int, k: int, d_ptr: int, i_ptr: int,
                      stream: int | None = None):
        _check(lib().vdb_ivf_search_device(self._h, ctypes.c_void_p(q_ptr), n, nprobe, k, ctypes.c_void_p(d_ptr),
                                           ctypes.c_void_p(i_ptr), ctypes.c_void_p(stream or 0)))

    def search_batch(self, queries, params, distances, indices):
        """search_batch (ivf_flat_index.h:55-58; declared, never defined in the reference)."""
        for q, p, d, i in zip(queries, params, distances, indices):
            D, I = self.search(q, p)
            d[...] = D.reshape(d.shape)
            i[...] = I.reshape(i.shape)

    # ---- persistence (IVFFlatIndex::save/load, ivf_flat_index.h:66-67) ----
    def save(self, path: str):
        _check(lib().vdb_ivf_save(self._h, os.fsencode(path)))

    def load(self, path: str):
        _check(lib().vdb_ivf_load(self._h, os.fsencode(path)))

    def get_dimension(self) -> int:
        return self.config.dimension

    # ---- sharding ----
    def set_shard(self, rank: int, world: int, owners=None):
        """Keep rank's lists of `world` (the LPT plan, or an explicit `owners` array)."""
        if owners is None:
            _check(lib().vdb_ivf_set_shard(self._h, rank, world))
        else:
            o = np.ascontiguousarray(owners, dtype=np.uint32)
            _check(lib().vdb_ivf_set_shard_owners(self._h, rank, world, _ptr(o)))

    def probe_census(self, rows_ptr: int, n: int, nprobe: int) -> np.ndarray:
        """Per list: how many of n device rows probe it (vdb_ivf_probe_census)."""
        out = np.empty(self.config.nlist, dtype=np.uint64)
        _check(lib().vdb_ivf_probe_census(self._h, ctypes.c_void_p(rows_ptr), n, nprobe, _ptr(out)))
        return out

    def attach_comm(self, comm_id: bytes, rank: int, world: int):
        """Join the RCCL communicator `comm_id` as `rank` of `world` (after set_shard /
        plan_shard with the same rank and world): searches then return final results."""
        if len(comm_id) != COMM_ID_BYTES:
            raise ValueError("comm_id must be COMM_ID_BYTES long")
        _check(lib().vdb_ivf_attach_comm(self._h, ctypes.c_char_p(comm_id), rank, world))

    def detach_comm(self):
        _check(lib().vdb_ivf_detach_comm(self._h))

    def comm_status(self):
        """(error message or None, exchanges issued, exchanges completed) of the attached
        communicator (vdb_ivf_comm_status)."""
        a, b = ctypes.c_uint64(0), ctypes.c_uint64(0)
        rc = lib().vdb_ivf_comm_status(self._h, ctypes.byref(a), ctypes.byref(b))
        return (lib().vdb_last_error().decode() if rc != 0 else None), a.value, b.value

    @property
    def group_size(self) -> int:
        return int(lib().vdb_ivf_group_size(self._h))

    def list_owners(self) -> np.ndarray:
        """Per list: the member (group) or rank (shard) storing it; 2**32 - 1 = none."""
        out = np.empty(self.config.nlist, dtype=np.uint32)
        _check(lib().vdb_ivf_list_owners(self._h, _ptr(out)))
        return out

    def plan_shard(self, rank: int, world: int, final_sizes, owners=None):
        """Sharded build: fix this rank's lists from the final list sizes before any add
        (the LPT plan, or an explicit `owners` array)."""
        s = np.ascontiguousarray(final_sizes, dtype=np.uint64)
        if len(s) != self.config.nlist:
            raise ValueError("final_sizes needs one entry per list")
        if owners is None:
            _check(lib().vdb_ivf_plan_shard(self._h, rank, world, _ptr(s)))
        else:
            o = np.ascontiguousarray(owners, dtype=np.uint32)
            _check(lib().vdb_ivf_plan_shard_owners(self._h, rank, world, _ptr(s), _ptr(o)))

    # ---- residency / stats ----
    def warmup_lists(self, list_ids):
        a = np.ascontiguousarray(list_ids, dtype=np.uint32)
        _check(lib().vdb_ivf_warmup(self._h, _ptr(a), len(a)))

    def evict_list(self, list_id: int):
        _check(lib().vdb_ivf_evict(self._h, list_id))

    def get_gpu_memory_usage(self) -> int:
        """Bytes of the GPU-resident lists, count * (dim * 4 + 8) each (ivf_flat_index.cpp:393-443)."""
        return int(lib().vdb_ivf_gpu_bytes(self._h))

    def gpu_bytes_allocated(self) -> int:
        """HBM really held for lists (padded 64-row blocks, whole cache in the tier) and centroids."""
        return int(lib().vdb_ivf_gpu_bytes_allocated(self._h))

    def get_total_vectors(self) -> int:
        return int(lib().vdb_ivf_ntotal(self._h))

    def list_sizes(self) -> np.ndarray:
        out = np.empty(self.config.nlist, dtype=np.uint64)
        _check(lib().vdb_ivf_list_sizes(self._h, _ptr(out)))
        return out

    def get_list(self, list_id: int):
        n = int(self.list_sizes()[list_id])
        v = np.empty((n, self.dimension), dtype=np.float32)
        i = np.empty(n, dtype=np.uint64)
        _check(lib().vdb_ivf_get_list(self._h, list_id, _ptr(v), _ptr(i)))
        return v, i

    def get_list_into(self, list_id: int, vectors: np.ndarray, ids: np.ndarray):
        """Copy list `list_id` into caller arrays (C-contiguous, sized count x dim / count)."""
        assert vectors.flags.c_contiguous and ids.flags.c_contiguous
        assert vectors.dtype == np.float32 and ids.dtype == np.uint64
        _check(lib().vdb_ivf_get_list(self._h, list_id, _ptr(vectors), _ptr(ids)))

    def set_batch(self, batch: int):
        _check(lib().vdb_ivf_set_batch(self._h, batch))

    def set_stale_slots(self, enable: bool):
        _check(lib().vdb_ivf_set_stale_slots(self._h, int(enable)))

    def set_coarse_mode(self, mode: int):
        """1: MFMA bounds + exact re-rank (default); 0: exact VALU coarse distances."""
        _check(lib().vdb_ivf_set_coarse_mode(self._h, mode))

    def set_option(self, name: str, value: int):
        """Engine option (vdb_ivf_set_option): tuning knobs and residency; never changes results."""
        _check(lib().vdb_ivf_set_option(self._h, name.encode(), int(value)))

    def coalesce_stats(self):
        """(device batches, search() calls served) of the host-API coalescing queue."""
        b, r = ctypes.c_uint64(0), ctypes.c_uint64(0)
        _check(lib().vdb_ivf_coalesce_stats(self._h, ctypes.byref(b), ctypes.byref(r)))
        return b.value, r.value

    def open_lists(self, path: str):
        """Serve the lists from an index file written by save() through the list-cache
        tier (set_option("list_cache_bytes", n) first); the handle becomes read-only."""
        _check(lib().vdb_ivf_open_lists(self._h, path.encode()))

    def cache_stats(self) -> dict:
        """List-cache tier counters (option list_cache_bytes; capacity 0 = tier off)."""
        st = CacheStats()
        _check(lib().vdb_ivf_cache_stats(self._h, ctypes.byref(st)))
        return st.as_dict()

    def fill_row_cache(self, weights=None):
        """Screened tier, file home: refill the row cache by expected survivor rows per vector
        (weights per list, e.g. survivor_histogram()) or by list size (None)."""
        if weights is None:
            _check(lib().vdb_ivf_fill_row_cache(self._h, None))
        else:
            c = np.ascontiguousarray(weights, dtype=np.uint64)
            if c.shape != (self.config.nlist,):
                raise ValueError("weights needs one entry per list")
            _check(lib().vdb_ivf_fill_row_cache(self._h, _ptr(c)))

    def survivor_histogram(self) -> np.ndarray:
        """Per list: the survivor rows the screened tier's batches needed so far."""
        out = np.zeros(self.config.nlist, dtype=np.uint64)
        _check(lib().vdb_ivf_survivor_histogram(self._h, _ptr(out)))
        return out

    def collect_stamps(self):
        """(option collect_stamps) the collect kernel's item timeline: (records [n, 4] uint64,
        wall clock Hz); resets the buffer."""
        n, hz = ctypes.c_uint64(0), ctypes.c_uint64(0)
        _check(lib().vdb_ivf_collect_stamps(self._h, None, 0, ctypes.byref(n), ctypes.byref(hz)))
        out = np.zeros((n.value, 4), dtype=np.uint64)
        if n.value:
            _check(lib().vdb_ivf_collect_stamps(self._h, out.ctypes.data, n.value, ctypes.byref(n), ctypes.byref(hz)))
        return out, hz.value

    def profile_enable(self, on: bool = True):
        _check(lib().vdb_ivf_profile_enable(self._h, int(on)))

    def profile_reset(self):
        _check(lib().vdb_ivf_profile_reset(self._h))

    def profile_read(self) -> dict:
        p = Profile()
        _check(lib().vdb_ivf_profile_read(self._h, ctypes.byref(p)))
        return p.as_dict()

    def synchronize(self):
        _check(lib().vdb_ivf_synchronize(self._h))

    @property
    def stream(self) -> int:
        return int(lib().vdb_ivf_stream(self._h) or 0)
