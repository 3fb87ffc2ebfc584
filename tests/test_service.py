"""CPU tests of the gRPC front end's contract (service.py): vdb.proto message shapes and the
request validation / response packing of QueryServiceImpl::Search
(server/query_service.cpp:68-168), exercised over a real localhost gRPC channel.

No GPU here, so the served index is a test double with the engine's search signature
(the GPU test in test_gpu_service.py serves the real engine)."""
import importlib

import grpc
import numpy as np
import pytest

from conftest import load_vdb

vdb = load_vdb()
service = importlib.import_module("vdb_amd.service")
M = service.messages()
U64MAX = np.iinfo(np.uint64).max


def test_message_fields_match_vdb_proto():
    # proto/vdb.proto:10-39
    def fields(name):
        return {f.name: (f.number, f.type, f.is_repeated) for f in M[name].DESCRIPTOR.fields}
    F = M["Vector"].DESCRIPTOR.fields[0].__class__
    assert fields("Vector") == {"id": (1, F.TYPE_UINT64, False), "values": (2, F.TYPE_FLOAT, True)}
    sr = fields("SearchRequest")
    assert [sr[n][0] for n in ("queries", "topk", "nprobe", "index", "metric", "rerank_exact")] == [1, 2, 3, 4, 5, 6]
    assert fields("Neighbor")["distance"][:2] == (2, F.TYPE_FLOAT)
    assert fields("SearchResponse")["results"][0] == 1
    req = M["SearchRequest"](topk=5, nprobe=3, index="x")
    req.queries.add(id=7, values=[1.0, 2.0])
    back = M["SearchRequest"].FromString(req.SerializeToString())
    assert back.queries[0].id == 7 and list(back.queries[0].values) == [1.0, 2.0] and back.topk == 5


class FakeIndex:
    """Test double: the engine's search signature, fixed answers, records its calls."""
    dimension = 4

    def __init__(self, fail=False):
        self.calls = []
        self.fail = fail
        self.warmed = []

    def search(self, q, nprobe, k):
        self.calls.append((q.copy(), nprobe, k))
        if self.fail:
            raise RuntimeError("device lost")
        D = np.tile(np.arange(k, dtype=np.float32), (q.shape[0], 1))
        I = np.tile(np.arange(100, 100 + k, dtype=np.uint64), (q.shape[0], 1))
        I[:, -1] = U64MAX                      # an unfilled slot: must not be sent
        D[:, -1] = np.finfo(np.float32).max
        return D, I

    def warmup_lists(self, lists):
        self.warmed.extend(lists)


@pytest.fixture()
def served():
    svc = service.QueryService()
    fake = FakeIndex()
    svc.register("idx", fake)
    svc.register("broken", FakeIndex(fail=True))
    server, port = service.make_server(svc, "127.0.0.1:0", workers=4)
    server.start()
    client = service.Client(f"127.0.0.1:{port}")
    yield client, fake
    client.close()
    server.stop(0)


def code_of(fn):
    with pytest.raises(grpc.RpcError) as e:
        fn()
    return e.value.code()


def test_validation_status_codes(served):
    c, _ = served
    q = np.ones((2, 4), np.float32)
    assert code_of(lambda: c.search(np.zeros((0, 4), np.float32), topk=5, index="idx")) == grpc.StatusCode.INVALID_ARGUMENT
    assert code_of(lambda: c.search(q, topk=0, index="idx")) == grpc.StatusCode.INVALID_ARGUMENT
    assert code_of(lambda: c.search(q, topk=1001, index="idx")) == grpc.StatusCode.INVALID_ARGUMENT
    assert code_of(lambda: c.search(q, topk=5, index="")) == grpc.StatusCode.INVALID_ARGUMENT
    assert code_of(lambda: c.search(q, topk=5, index="nope")) == grpc.StatusCode.NOT_FOUND
    assert code_of(lambda: c.search(np.ones((2, 3), np.float32), topk=5, index="idx")) == grpc.StatusCode.INVALID_ARGUMENT
    assert code_of(lambda: c.search(q, topk=5, index="broken")) == grpc.StatusCode.INTERNAL


def test_search_packing_and_defaults(served):
    c, fake = served
    q = np.arange(8, dtype=np.float32).reshape(2, 4)
    resp = c.search(q, topk=5, nprobe=0, index="idx", metric="InnerProduct")
    assert len(resp.results) == 2
    for r in resp.results:
        assert [n.id for n in r.neighbors] == [100, 101, 102, 103]      # the UINT64_MAX slot is skipped
        assert [n.distance for n in r.neighbors] == [0.0, 1.0, 2.0, 3.0]
    sent_q, nprobe, k = fake.calls[-1]
    assert nprobe == 8 and k == 5                                        # nprobe <= 0 -> 8
    assert np.array_equal(sent_q, q)
    c.search(q, topk=1000, nprobe=3, index="idx")
    assert fake.calls[-1][1:] == (3, 1000)


def test_warmup(served):
    c, fake = served
    c.warmup("idx", [3, -1, 5])
    assert fake.warmed == [3, 5]                                         # negative ids skipped
    assert code_of(lambda: c.warmup("nope", [1])) == grpc.StatusCode.NOT_FOUND


def test_load_index_missing_epoch(tmp_path):
    svc = service.QueryService(str(tmp_path))
    st, _, _ = svc.load_index(M["LoadIndexRequest"](index="a", epoch="e1"))
    assert st == "NOT_FOUND"
    assert service.QueryService().load_index(M["LoadIndexRequest"](index="a", epoch="e1"))[0] == "FAILED_PRECONDITION"


def test_cli_accepts_both_flag_forms(monkeypatch):
    seen = {}

    def fake_make_server(svc, address, workers):
        seen["address"], seen["workers"], seen["data"] = address, workers, svc.data_path
        raise SystemExit(0)

    monkeypatch.setattr(service, "make_server", fake_make_server)
    with pytest.raises(SystemExit):
        service.main(["--address=127.0.0.1:6000", "--data-path", "/tmp/x", "--workers=3", "--batch-size=64",
                      "--coalesce-window", "2"])
    assert seen == {"address": "127.0.0.1:6000", "workers": 3, "data": "/tmp/x"}


def test_load_index_rejects_paths_outside_data_path(tmp_path):
    # LoadIndex builds <data_path>/<index>/<epoch>; a network caller must not be able to
    # name a file outside --data-path (query_service.cpp:218-265 concatenates unchecked)
    (tmp_path / "outside.json").write_text('{"dimension": 4, "nlist": 1}')
    svc = service.QueryService(str(tmp_path / "data"))
    for index, epoch in (("..", "outside"), ("a/../..", "outside"), ("/etc", "passwd"), ("idx", "../../outside"),
                         ("", "e"), ("idx", "")):
        st, detail, _ = svc.load_index(M["LoadIndexRequest"](index=index, epoch=epoch))
        assert st == "INVALID_ARGUMENT", (index, epoch, st, detail)
    st, _, _ = svc.load_index(M["LoadIndexRequest"](index="idx", epoch="e1"))
    assert st == "NOT_FOUND"
