"""CPU tests of the drop-in boundary: the C ABI library loads, exports every entry
point include/vdb_ivf.h declares, carries gfx950 code, the C++ surface exports the
reference class methods, and host-only logic (shard planning) behaves. No kernel is
launched here (no GPU in this container)."""
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import PKG_DIR, ROOT, load_vdb

vdb = load_vdb()
HEADER = os.path.join(ROOT, "include", "vdb_ivf.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(vdb_\w+)\s*\(", text)))


def test_every_declared_symbol_is_exported():
    names = declared_functions()
    assert len(names) >= 30
    lib = vdb.lib()
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    out = subprocess.check_output(["nm", "-D", "--defined-only", vdb.LIB_PATH], text=True)
    exported = set(re.findall(r" T (vdb_\w+)", out))
    assert set(names) <= exported


def test_library_carries_gfx950_code_object():
    data = open(vdb.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data
    out = subprocess.check_output(["readelf", "-d", vdb.LIB_PATH], text=True)
    assert "libtorch" not in out and "libc10" not in out, "no torch types or libraries at the boundary"


def test_cpp_surface_exports_reference_methods():
    out = subprocess.check_output(["nm", "-DC", "--defined-only", vdb.CPP_LIB_PATH], text=True)
    for m in ["vdb::IVFFlatIndex::IVFFlatIndex(", "vdb::IVFFlatIndex::train(", "vdb::IVFFlatIndex::add(",
              "vdb::IVFFlatIndex::search(", "vdb::IVFFlatIndex::search_batch(", "vdb::IVFFlatIndex::warmup_lists(",
              "vdb::IVFFlatIndex::evict_list(", "vdb::IVFFlatIndex::get_gpu_memory_usage()",
              "vdb::IVFFlatIndex::get_total_vectors()", "vdb::IVFFlatIndex::save(", "vdb::IVFFlatIndex::load(",
              "vdb::TransferManager::allocate_pinned(", "vdb::TransferManager::allocate_device(",
              "vdb::TransferManager::enqueue_transfer(", "vdb::TransferManager::get_stream()",
              "vdb::TransferManager::synchronize()", "vdb::TransferManager::get_memory_stats()"]:
        assert m in out, m


def test_cpp_header_needs_no_device_headers():
    src = "#include \"vdb/ivf_flat_index.h\"\nint main(){vdb::IVFFlatIndex::Config c{64,16,vdb::kernels::Metric::L2};return (int)c.nlist-16;}\n"
    p = subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-I", os.path.join(ROOT, "include"), "-x", "c++", "-"],
                       input=src, text=True, capture_output=True)
    assert p.returncode == 0, p.stderr


def test_metric_ordinals_match_reference():
    assert (int(vdb.Metric.L2), int(vdb.Metric.InnerProduct), int(vdb.Metric.Cosine)) == (0, 1, 2)


def test_shard_plan_is_lpt_and_deterministic():
    rng = np.random.default_rng(0)
    sizes = rng.integers(0, 50000, 4096).astype(np.uint64)
    for world in (1, 2, 4, 8):
        owner = vdb.shard_plan(sizes, world)
        assert np.array_equal(owner, vdb.shard_plan(sizes, world))
        assert owner.max() < world
        loads = np.bincount(owner, weights=sizes.astype(np.float64), minlength=world)
        # LPT bound: max load <= mean + largest item
        assert loads.max() <= loads.mean() + sizes.max()
    assert np.array_equal(vdb.shard_plan(np.array([5, 3, 9, 1, 7, 7], np.uint64), 2), [0, 0, 0, 1, 1, 1])


def test_config_validation_matches_reference():
    with pytest.raises(ValueError):
        vdb.IVFFlatIndex(vdb.IVFFlatIndex.Config(0, 16))
    with pytest.raises(ValueError):
        vdb.IVFFlatIndex(vdb.IVFFlatIndex.Config(64, 0))


def test_no_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    with pytest.raises(vdb.VdbError):
        vdb.IVFFlatIndex(vdb.IVFFlatIndex.Config(8, 4))
    assert vdb.lib().vdb_ivf_ntotal(None) == 0


def test_product_never_imports_the_oracle():
    for dirpath, _, files in os.walk(PKG_DIR):
        for f in files:
            if f.endswith((".py", ".cpp", ".hip", ".hpp", ".h")):
                text = open(os.path.join(dirpath, f), errors="ignore").read()
                assert "import oracle" not in text and "cpu_ref" not in text and "oracle_" not in text, f


def test_probe_weighted_plan_balances_popular_lists():
    """vdb_shard_plan_probe_weighted: the same lists and sizes, but one list probed by
    every query: the size-only LPT puts it with as many vectors as the others, the
    probe-weighted LPT gives its rank fewer vectors. Deterministic; every list owned."""
    sizes = np.array([1000, 1000, 1000, 1000, 500, 500, 500, 500], dtype=np.uint64)
    counts = np.array([64000, 10, 10, 10, 10, 10, 10, 10], dtype=np.uint64)  # list 0: a hub
    lpt = vdb.shard_plan(sizes, 2)
    w = vdb.shard_plan_probe_weighted(sizes, counts, 64000, 64, 2)
    assert np.array_equal(w, vdb.shard_plan_probe_weighted(sizes, counts, 64000, 64, 2))
    assert set(w.tolist()) == {0, 1} and set(lpt.tolist()) == {0, 1}
    vec = lambda o, r: int(sizes[o == r].sum())
    assert vec(lpt, lpt[0]) == vec(lpt, 1 - lpt[0])          # sizes balanced, hub ignored
    assert vec(w, w[0]) < vec(w, 1 - w[0])                    # the hub's rank holds fewer vectors
    # uniform popularity: the weighted plan balances sizes like the LPT
    uni = np.full(8, 640, dtype=np.uint64)
    wu = vdb.shard_plan_probe_weighted(sizes, uni, 64000, 64, 2)
    assert vec(wu, 0) == vec(wu, 1)
