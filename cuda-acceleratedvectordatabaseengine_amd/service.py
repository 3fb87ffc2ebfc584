"""gRPC front end: ``vdb.QueryService`` (reference ``proto/vdb.proto:89-97``) over the engine.

The reference server (``server/query_service.cpp``, ``server/main.cpp``) is C++ gRPC; this
image has no C++ gRPC or ``protoc``, so the same wire contract is served with the Python
``grpc`` runtime and message classes built from a descriptor written out below (field names,
numbers and types exactly as ``proto/vdb.proto``). The search itself is the engine's
thread-safe host API: concurrent handlers' calls are coalesced into shared device batches
inside ``libvdb_ivf.so`` (``vdb_ivf_search``), each call keeping its own exact result.

Behaviour follows ``QueryServiceImpl::Search`` (query_service.cpp:68-168):
  * no queries -> INVALID_ARGUMENT; ``topk`` outside [1, 1000] -> INVALID_ARGUMENT;
    empty index name -> INVALID_ARGUMENT; unknown index -> NOT_FOUND;
  * ``nprobe <= 0`` -> 8; the ``metric`` string is parsed and ignored (the index's
    build-time metric wins); ``rerank_exact`` is ignored (A7);
  * a query whose length differs from the index dimension -> INVALID_ARGUMENT;
  * results skip ``UINT64_MAX`` slots (query_service.cpp:150); engine errors -> INTERNAL.
``Warmup`` (170-204): unknown index -> NOT_FOUND; negative list ids are skipped.
``LoadIndex`` (206-265): loads ``<data_path>/<index>/<epoch>.ivf`` (``vdb_ivf_save`` files,
with ``<epoch>.json`` holding dimension / nlist / metric) and makes it the served index.

CLI flags mirror ``server/main.cpp:131-176`` (``--address --data-path --gpu-memory
--batch-size --coalesce-window``) and accept both ``--flag value`` and ``--flag=value``
(the reference's runner scripts pass the second form, which its parser rejected).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
from concurrent import futures

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))

UINT64_MAX = np.iinfo(np.uint64).max


# ---------------------------------------------------------------------------
# vdb.proto messages (proto/vdb.proto:10-87), built without protoc
# ---------------------------------------------------------------------------
def _build_messages():
    from google.protobuf import descriptor_pb2, descriptor_pool, message_factory
    from google.protobuf import empty_pb2  # noqa: F401  (registers google/protobuf/empty.proto)

    F = descriptor_pb2.FieldDescriptorProto
    fdp = descriptor_pb2.FileDescriptorProto(name="vdb.proto", package="vdb", syntax="proto3")
    fdp.dependency.append("google/protobuf/empty.proto")

    def msg(name, *fields):
        m = fdp.message_type.add(name=name)
        for fname, num, ftype, label, tname in fields:
            f = m.field.add(name=fname, number=num, type=ftype, label=label)
            if tname:
                f.type_name = tname
        return m

    opt, rep = F.LABEL_OPTIONAL, F.LABEL_REPEATED
    msg("Vector", ("id", 1, F.TYPE_UINT64, opt, None), ("values", 2, F.TYPE_FLOAT, rep, None))
    msg("SearchRequest", ("queries", 1, F.TYPE_MESSAGE, rep, ".vdb.Vector"), ("topk", 2, F.TYPE_INT32, opt, None),
        ("nprobe", 3, F.TYPE_INT32, opt, None), ("index", 4, F.TYPE_STRING, opt, None),
        ("metric", 5, F.TYPE_STRING, opt, None), ("rerank_exact", 6, F.TYPE_BOOL, opt, None))
    msg("Neighbor", ("id", 1, F.TYPE_UINT64, opt, None), ("distance", 2, F.TYPE_FLOAT, opt, None))
    msg("SearchResult", ("neighbors", 1, F.TYPE_MESSAGE, rep, ".vdb.Neighbor"))
    msg("SearchResponse", ("results", 1, F.TYPE_MESSAGE, rep, ".vdb.SearchResult"))
    msg("WarmupRequest", ("index", 1, F.TYPE_STRING, opt, None), ("lists", 2, F.TYPE_INT32, rep, None))
    msg("LoadIndexRequest", ("index", 1, F.TYPE_STRING, opt, None), ("epoch", 2, F.TYPE_STRING, opt, None))
    msg("StatsRequest", ("index", 1, F.TYPE_STRING, opt, None))
    msg("StatsResponse", ("total_vectors", 1, F.TYPE_UINT64, opt, None), ("indexed_vectors", 2, F.TYPE_UINT64, opt, None),
        ("current_epoch", 3, F.TYPE_STRING, opt, None), ("gpu_memory_used", 4, F.TYPE_FLOAT, opt, None),
        ("nvme_usage", 5, F.TYPE_FLOAT, opt, None))
    pool = descriptor_pool.DescriptorPool()
    from google.protobuf import empty_pb2 as _e
    pool.AddSerializedFile(_e.DESCRIPTOR.serialized_pb)
    pool.Add(fdp)
    names = ["Vector", "SearchRequest", "Neighbor", "SearchResult", "SearchResponse", "WarmupRequest",
             "LoadIndexRequest", "StatsRequest", "StatsResponse"]
    classes = {n: message_factory.GetMessageClass(pool.FindMessageTypeByName("vdb." + n)) for n in names}
    classes["Empty"] = message_factory.GetMessageClass(pool.FindMessageTypeByName("google.protobuf.Empty"))
    return classes


_MESSAGES = None
_MSG_LOCK = threading.Lock()


def messages():
    """The vdb.proto message classes (``messages()["SearchRequest"]`` etc.)."""
    global _MESSAGES
    with _MSG_LOCK:
        if _MESSAGES is None:
            _MESSAGES = _build_messages()
        return _MESSAGES


# ---------------------------------------------------------------------------
# QueryService
# ---------------------------------------------------------------------------
class QueryService:
    """vdb.QueryService over named indexes (query_service.h:23-128, Search/Warmup/LoadIndex)."""

    def __init__(self, data_path: str | None = None, device: int = 0):
        self.data_path = data_path
        self.device = device
        self._indexes = {}  # name -> (index, epoch)
        self._lock = threading.RLock()  # the reference's shared_mutex over the index map (212-216)

    # registry ----------------------------------------------------------------
    def register(self, name: str, index, epoch: str = "") -> None:
        with self._lock:
            self._indexes[name] = (index, epoch)

    def get_index(self, name: str):
        with self._lock:
            entry = self._indexes.get(name)
        return entry[0] if entry else None

    # Search (query_service.cpp:68-168) ---------------------------------------
    def search(self, request):
        """Returns (status_name, detail, response-or-None); status_name is a grpc.StatusCode name."""
        M = messages()
        if len(request.queries) == 0:
            return "INVALID_ARGUMENT", "No queries provided", None
        if request.topk <= 0 or request.topk > 1000:
            return "INVALID_ARGUMENT", "Invalid topk value", None
        if not request.index:
            return "INVALID_ARGUMENT", "Index name required", None
        index = self.get_index(request.index)
        if index is None:
            return "NOT_FOUND", "Index not found: " + request.index, None
        k = int(request.topk)
        nprobe = int(request.nprobe) if request.nprobe > 0 else 8
        dim = index.dimension
        q = np.empty((len(request.queries), dim), dtype=np.float32)
        for i, v in enumerate(request.queries):
            if len(v.values) != dim:
                return "INVALID_ARGUMENT", "Query dimension mismatch", None
            q[i] = v.values
        try:
            D, I = index.search(q, nprobe=nprobe, k=k)
        except Exception as e:  # engine failure -> INTERNAL (164-167)
            return "INTERNAL", "Search failed: " + str(e), None
        resp = M["SearchResponse"]()
        for qi in range(q.shape[0]):
            res = resp.results.add()
            keep = I[qi] != UINT64_MAX
            for nid, d in zip(I[qi][keep].tolist(), D[qi][keep].tolist()):
                res.neighbors.add(id=nid, distance=d)
        return "OK", "", resp

    # Warmup (170-204) ------------------------------------------------------------
    def warmup(self, request):
        index = self.get_index(request.index)
        if index is None:
            return "NOT_FOUND", "Index not found: " + request.index, None
        try:
            lists = [l for l in request.lists if l >= 0]
            if lists:
                index.warmup_lists(lists)
        except Exception as e:
            return "INTERNAL", "Warmup failed: " + str(e), None
        return "OK", "", messages()["Empty"]()

    # LoadIndex (206-265) -------------------------------------------------------
    def load_index(self, request):
        if not self.data_path:
            return "FAILED_PRECONDITION", "server has no data path", None
        # names are single path components: no separators, no '..', nothing that
        # resolves outside --data-path (the reference concatenates them unchecked)
        for part in (request.index, request.epoch):
            if not part or part in (".", "..") or "/" in part or "\\" in part or "\0" in part:
                return "INVALID_ARGUMENT", "index and epoch must be plain names", None
        root = os.path.realpath(self.data_path)
        base = os.path.join(root, request.index, request.epoch)
        if os.path.commonpath([root, os.path.realpath(base + ".ivf")]) != root:
            return "INVALID_ARGUMENT", "index path leaves the data path", None
        try:
            with open(base + ".json") as f:
                meta = json.load(f)
        except OSError:
            return "NOT_FOUND", f"Epoch not found: {request.index}/{request.epoch}", None
        try:
            from . import IVFFlatIndex, Metric  # the package this module ships in
        except ImportError:
            vdb = sys.modules.get("vdb_amd")
            IVFFlatIndex, Metric = vdb.IVFFlatIndex, vdb.Metric
        try:
            idx = IVFFlatIndex(IVFFlatIndex.Config(int(meta["dimension"]), int(meta["nlist"]),
                                                   Metric(int(meta.get("metric", 0))), device=self.device))
            idx.load(base + ".ivf")
        except Exception as e:
            return "INTERNAL", "Load failed: " + str(e), None
        self.register(request.index, idx, request.epoch)
        return "OK", "", messages()["Empty"]()


def save_epoch(index, data_path: str, name: str, epoch: str) -> str:
    """Write an index as ``<data_path>/<name>/<epoch>.ivf`` (+ ``.json``) for LoadIndex."""
    d = os.path.join(data_path, name)
    os.makedirs(d, exist_ok=True)
    base = os.path.join(d, epoch)
    index.save(base + ".ivf")
    with open(base + ".json", "w") as f:
        json.dump({"dimension": index.dimension, "nlist": index.config.nlist, "metric": int(index.config.metric)}, f)
    return base


# ---------------------------------------------------------------------------
# gRPC plumbing
# ---------------------------------------------------------------------------
def _handler(fn, req_cls, resp_cls):
    import grpc

    def call(request, context):
        status, detail, resp = fn(request)
        if status != "OK":
            context.abort(getattr(grpc.StatusCode, status), detail)
        return resp

    return grpc.unary_unary_rpc_method_handler(call, request_deserializer=req_cls.FromString,
                                               response_serializer=resp_cls.SerializeToString)


def make_server(service: QueryService, address: str, workers: int = 32):
    """A grpc.Server serving vdb.QueryService at `address` (not started)."""
    import grpc
    M = messages()
    handlers = grpc.method_handlers_generic_handler("vdb.QueryService", {
        "Search": _handler(service.search, M["SearchRequest"], M["SearchResponse"]),
        "Warmup": _handler(service.warmup, M["WarmupRequest"], M["Empty"]),
        "LoadIndex": _handler(service.load_index, M["LoadIndexRequest"], M["Empty"]),
    })
    # the reference: sync server, 4 CQs, 2-8 pollers (main.cpp:92-94); here a thread pool
    server = grpc.server(futures.ThreadPoolExecutor(max_workers=workers),
                         options=[("grpc.max_receive_message_length", 256 << 20),
                                  ("grpc.max_send_message_length", 256 << 20)])
    server.add_generic_rpc_handlers((handlers,))
    port = server.add_insecure_port(address)
    return server, port


class Client:
    """Minimal vdb.QueryService client (what grpc_integration_test.cpp / load_test.cpp use)."""

    def __init__(self, target: str):
        import grpc
        M = messages()
        self.channel = grpc.insecure_channel(target)
        self._search = self.channel.unary_unary("/vdb.QueryService/Search",
                                                request_serializer=M["SearchRequest"].SerializeToString,
                                                response_deserializer=M["SearchResponse"].FromString)
        self._warmup = self.channel.unary_unary("/vdb.QueryService/Warmup",
                                                request_serializer=M["WarmupRequest"].SerializeToString,
                                                response_deserializer=M["Empty"].FromString)
        self._load = self.channel.unary_unary("/vdb.QueryService/LoadIndex",
                                              request_serializer=M["LoadIndexRequest"].SerializeToString,
                                              response_deserializer=M["Empty"].FromString)

    def search_request(self, queries, topk=10, nprobe=0, index="", metric="L2"):
        M = messages()
        req = M["SearchRequest"](topk=topk, nprobe=nprobe, index=index, metric=metric)
        for i, q in enumerate(np.asarray(queries, dtype=np.float32)):
            req.queries.add(id=i, values=np.ravel(q).tolist())
        return req

    def search(self, queries, topk=10, nprobe=0, index="", metric="L2", timeout=60.0):
        return self._search(self.search_request(queries, topk, nprobe, index, metric), timeout=timeout)

    def warmup(self, index, lists=(), timeout=60.0):
        return self._warmup(messages()["WarmupRequest"](index=index, lists=list(lists)), timeout=timeout)

    def load_index(self, index, epoch, timeout=600.0):
        return self._load(messages()["LoadIndexRequest"](index=index, epoch=epoch), timeout=timeout)

    def close(self):
        self.channel.close()


def main(argv=None):
    ap = argparse.ArgumentParser(description="vdb.QueryService on an MI355X (server/main.cpp flags)")
    ap.add_argument("--address", default="0.0.0.0:50051")
    ap.add_argument("--data-path", default="/data/vdb")
    ap.add_argument("--gpu-memory", type=float, default=0.0, help="GB (accepted; the index stays HBM-resident)")
    ap.add_argument("--batch-size", type=int, default=1024, help="max queries per coalesced device batch")
    ap.add_argument("--coalesce-window", type=float, default=0.0, help="ms to wait for more calls (0: none)")
    ap.add_argument("--index", action="append", default=[], metavar="NAME=EPOCH", help="load at startup")
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--workers", type=int, default=32)
    args = ap.parse_args(argv)
    # validation as main.cpp:179-187
    if args.batch_size <= 0 or args.coalesce_window < 0 or args.gpu_memory < 0:
        ap.error("invalid batch size, coalesce window or GPU memory")
    svc = QueryService(args.data_path, args.device)
    M = messages()
    for spec in args.index:
        name, epoch = spec.split("=", 1)
        st, detail, _ = svc.load_index(M["LoadIndexRequest"](index=name, epoch=epoch))
        if st != "OK":
            print(f"failed to load {spec}: {detail}", file=sys.stderr)
            return 1
        idx = svc.get_index(name)
        idx.set_option("coalesce_max_queries", args.batch_size)
        idx.set_option("coalesce_window_us", int(args.coalesce_window * 1000))
    server, port = make_server(svc, args.address, args.workers)
    server.start()
    print(f"vdb.QueryService listening on {args.address} (port {port})", flush=True)
    server.wait_for_termination()
    return 0


if __name__ == "__main__":
    sys.exit(main())
