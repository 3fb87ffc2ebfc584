#!/usr/bin/env python3
"""Closed-loop load test of vdb.QueryService/Search (the reference's
test/integration/load_test.cpp: N client threads, Q queries per request, nprobe 8, top-k,
random N(0,1) queries) against service.py serving the engine on cuda:0.

Clients run in separate processes (the server process keeps its own GIL for the gRPC
handlers). Reports requests/s, queries/s and p50/p99 request latency, with the engine's
request coalescing on and off, one JSON line per mode.

usage: python tools/grpc_load.py [--nvec 1000000 --dim 128 --nlist 1024 --procs 4 --threads 8
                                  --seconds 10 --queries-per-request 1 --topk 10]
"""
import argparse
import importlib.util
import json
import multiprocessing as mp
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "cuda-acceleratedvectordatabaseengine_amd")


def load_pkg():
    spec = importlib.util.spec_from_file_location("vdb_amd", os.path.join(PKG, "__init__.py"),
                                                  submodule_search_locations=[PKG])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["vdb_amd"] = mod
    spec.loader.exec_module(mod)
    return mod, importlib.import_module("vdb_amd.service")


def client_proc(target, threads, seconds, qpr, dim, topk, seed, out_q):
    import threading
    _, service = load_pkg()
    lat, errs = [], [0]
    stop_at = time.perf_counter() + seconds

    def run(t):
        c = service.Client(target)
        rng = np.random.default_rng(seed * 1000 + t)
        while time.perf_counter() < stop_at:
            q = rng.standard_normal((qpr, dim)).astype(np.float32)
            t0 = time.perf_counter()
            try:
                c.search(q, topk=topk, nprobe=8, index="test_index", timeout=10.0)
                lat.append(time.perf_counter() - t0)
            except Exception:
                errs[0] += 1
        c.close()

    ths = [threading.Thread(target=run, args=(t,)) for t in range(threads)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    out_q.put((lat, errs[0]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nvec", type=int, default=1_000_000)
    ap.add_argument("--dim", type=int, default=128)
    ap.add_argument("--nlist", type=int, default=1024)
    ap.add_argument("--procs", type=int, default=4)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--seconds", type=float, default=8.0)
    ap.add_argument("--queries-per-request", type=int, default=1)
    ap.add_argument("--topk", type=int, default=10)
    ap.add_argument("--workers", type=int, default=32)
    args = ap.parse_args()

    import torch
    vdb, service = load_pkg()
    dev = torch.device("cuda", 0)
    with torch.cuda.stream(torch.cuda.Stream(dev)):
        s = torch.cuda.current_stream().cuda_stream
        data = torch.empty((args.nvec, args.dim), dtype=torch.float32, device=dev)
        vdb.gen_normal_device(data.data_ptr(), args.nvec * args.dim, seed=12345, stream=s)
        ids = torch.arange(args.nvec, dtype=torch.int64, device=dev)
        torch.cuda.synchronize()
        idx = vdb.IVFFlatIndex(vdb.IVFFlatIndex.Config(args.dim, args.nlist))
        idx.train_device(data.data_ptr(), min(100_000, args.nvec))
        idx.add_device(data.data_ptr(), ids.data_ptr(), args.nvec)
        del data, ids
        torch.cuda.synchronize()
    svc = service.QueryService()
    svc.register("test_index", idx)
    server, port = service.make_server(svc, "127.0.0.1:0", workers=args.workers)
    server.start()
    target = f"127.0.0.1:{port}"
    service.Client(target).search(np.zeros((1, args.dim), np.float32), topk=args.topk, nprobe=8,
                                  index="test_index")  # warm-up
    ctx = mp.get_context("spawn")
    for coalesce in (1, 0):
        idx.set_option("coalesce", coalesce)
        b0 = idx.coalesce_stats()
        q = ctx.Queue()
        procs = [ctx.Process(target=client_proc, args=(target, args.threads, args.seconds, args.queries_per_request,
                                                       args.dim, args.topk, p, q)) for p in range(args.procs)]
        t0 = time.perf_counter()
        for p in procs:
            p.start()
        lats, errs = [], 0
        for _ in procs:
            l, e = q.get()
            lats += l
            errs += e
        for p in procs:
            p.join()
        wall = time.perf_counter() - t0
        b1 = idx.coalesce_stats()
        lats.sort()
        pct = lambda p: lats[int(p * (len(lats) - 1))] * 1e3 if lats else 0.0  # query_service.cpp:790-798
        batches, served = b1[0] - b0[0], b1[1] - b0[1]
        print(json.dumps({
            "metric": "vdb.QueryService/Search closed-loop load (load_test.cpp shape)",
            "coalesce": bool(coalesce), "clients": args.procs * args.threads,
            "queries_per_request": args.queries_per_request, "requests": len(lats), "errors": errs,
            "requests_per_s": round(len(lats) / args.seconds, 1),
            "queries_per_s": round(len(lats) * args.queries_per_request / args.seconds, 1),
            "p50_ms": round(pct(0.5), 3), "p99_ms": round(pct(0.99), 3),
            "device_batches": batches, "calls_per_device_batch": round(served / batches, 2) if batches else None,
            "index": f"{args.nvec}x{args.dim} nlist {args.nlist}, nprobe 8, k {args.topk}",
            "wall_s": round(wall, 2)}), flush=True)
    server.stop(0)


if __name__ == "__main__":
    main()
