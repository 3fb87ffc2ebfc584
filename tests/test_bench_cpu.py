"""CPU: bench.py's host logic that needs no GPU — the PMC traffic lookup tied to the
library's build id (a traffic figure measured on other kernel sources must not reach the
bench line), and the per-rank balance summary."""
import importlib.util
import json
import os

from conftest import ROOT, load_vdb

vdb = load_vdb()


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_traffic_lookup_requires_the_same_build(tmp_path):
    bench = _bench()
    key = "10000000x768/4096/32/64/10/N1"
    bid = vdb.build_id()
    assert len(bid) == 16 and bid != "unknown"
    p = tmp_path / "traffic.json"
    p.write_text(json.dumps({"workloads": {key: {"workload": key, "build_id": bid, "hbm_bytes_per_scan_launch": 123}}}))
    assert bench.lookup_traffic(str(p), key, bid)[0] == 123
    t, note = bench.lookup_traffic(str(p), key, "0" * 16)   # measured on another build: stale
    assert t is None and "measured on build" in note
    p.write_text(json.dumps({"workloads": {key: {"workload": key, "hbm_bytes_per_scan_launch": 123}}}))
    assert bench.lookup_traffic(str(p), key, bid)[0] is None  # unstamped entries are never used
    assert bench.lookup_traffic(str(p), key + "/mixture", bid)[0] is None
    assert bench.lookup_traffic(str(tmp_path / "missing.json"), key, bid)[0] is None


def test_rank_balance_summary():
    bench = _bench()
    ranks = [{"rank": r, "scan_ms": 1.0 + 0.1 * r, "search_ms": 2.0, "ms_per_step": 1.5 - 0.1 * r,
              "scan_bytes_per_batch": 100 + r} for r in range(4)]
    b = bench.balance(ranks)
    assert b["scan_ms"]["argmax_rank"] == 3 and abs(b["scan_ms"]["max_over_min"] - 1.3) < 1e-9
    assert b["ms_per_step"]["argmax_rank"] == 0
    assert b["search_ms"]["max_over_min"] == 1.0
