// group.cpp — multi-GPU forms of the IVF-Flat search path.
//
// The reference searches on the implicit device 0 only (ivf_flat_index.cpp:214-255; its
// README's "Multi-GPU Support" has no code behind it). Here an index is sharded by
// inverted list across GPUs and every search batch ends in ONE RCCL all-gather (over
// xGMI) of each GPU's packed partial top-k, then the on-device unique-id merge; the
// result is bit-identical to one GPU (unique-id top-k of a union = unique-id top-k of
// the per-part unique-id top-k, under the (dist, id) order of merge_results,
// cpp:474-518). Two deployments share the exchange code in engine.hpp:
//
//  * one process per GPU (vdb_ivf_attach_comm): each process holds one shard
//    (set_shard / plan_shard) and a communicator from ncclCommInitRank;
//  * one process driving every GPU (vdb_ivf_create_group): one member handle per device
//    and ncclCommInitAll. The group is a vdb_ivf* like any other, so the C++ drop-in
//    (vdb::IVFFlatIndex), the coalescing host API and the gRPC service serve a sharded
//    index unchanged. Lists are placed on members when they first receive vectors,
//    largest first on the least-loaded member (for a bulk add this is exactly the LPT
//    plan of vdb_shard_plan), and stay there.
#include "engine.hpp"

#include <set>

namespace vdbe {
namespace {

// The ABI calls switch devices; the caller's current device is restored on return.
struct DeviceGuard {
    int prev = 0;
    DeviceGuard() { (void)hipGetDevice(&prev); }
    ~DeviceGuard() { (void)hipSetDevice(prev); }
};

// Rows per build chunk: at most 8 GiB of padded rows on a device at a time.
uint64_t chunk_rows(uint32_t dp) { return std::max<uint64_t>(1, (8ull << 30) / ((uint64_t)dp * 4)); }

// Run f(m) for every member on its own thread (members are independent devices);
// the first exception is rethrown after every thread has finished.
template <class F>
void for_members(vdb_ivf* g, F&& f) {
    const size_t M = g->members.size();
    if (M == 1) {
        g->members[0]->set_device();
        f(0);
        return;
    }
    std::vector<std::exception_ptr> err(M);
    std::vector<std::thread> th;
    for (size_t m = 0; m < M; ++m)
        th.emplace_back([&, m] {
            try {
                g->members[m]->set_device();
                f(m);
            } catch (...) {
                err[m] = std::current_exception();
            }
        });
    for (auto& t : th) t.join();
    for (auto& e : err)
        if (e) std::rethrow_exception(e);
}

// The group's own copies of the global list state (every member counts every list).
void sync_counts(vdb_ivf* g) {
    g->count = g->members[0]->count;
    g->total = g->members[0]->total;
}

// Place the lists that receive their first vectors: largest first, each on the member
// holding the fewest vectors (lowest member on ties), then relayout every member.
void place(vdb_ivf* g, const uint32_t* asg, uint64_t n) {
    const uint32_t L = g->nlist, M = (uint32_t)g->members.size();
    std::vector<uint64_t> added(L, 0);
    for (uint64_t i = 0; i < n; ++i) added[asg[i]]++;
    const std::vector<uint64_t>& cnt = g->members[0]->count;
    std::vector<uint64_t> load(M, 0);
    std::vector<uint32_t> fresh;
    for (uint32_t l = 0; l < L; ++l) {
        if (g->owner[l] != vdb_ivf::kUnplaced) load[g->owner[l]] += cnt[l];
        else if (added[l]) fresh.push_back(l);
    }
    if (fresh.empty()) return;
    std::stable_sort(fresh.begin(), fresh.end(), [&](uint32_t a, uint32_t b) { return added[a] > added[b]; });
    for (uint32_t l : fresh) {
        uint32_t best = 0;
        for (uint32_t m = 1; m < M; ++m)
            if (load[m] < load[best]) best = m;
        g->owner[l] = best;
        load[best] += added[l];
    }
    for_members(g, [&](size_t m) {
        std::vector<uint8_t> own(L);
        for (uint32_t l = 0; l < L; ++l) own[l] = g->owner[l] == m;
        g->members[m]->set_owned(own);
    });
}

void broadcast_centroids(vdb_ivf* g) {
    std::vector<float> c((size_t)g->nlist * g->dim);
    g->members[0]->set_device();
    g->members[0]->export_centroids(c.data());
    for (size_t m = 1; m < g->members.size(); ++m) {
        g->members[m]->set_device();
        g->members[m]->set_centroids_host(c.data());
    }
}

}  // namespace

namespace group {

void train_device(vdb_ivf* g, const float* d_v, uint64_t n) {
    DeviceGuard dg;
    g->members[0]->set_device();
    g->members[0]->train(d_v, n);
    broadcast_centroids(g);
}

void set_centroids(vdb_ivf* g, const float* c) {
    DeviceGuard dg;
    for (auto& mb : g->members) {
        mb->set_device();
        mb->set_centroids_host(c);
    }
}

// add / add_to_lists from host rows: exact assignment on member 0 (unless the lists
// are given), placement, then every member appends the rows of its lists (each member
// reads the whole input and keeps the rows it stores; the others are counted).
void add_host(vdb_ivf* g, const float* v, const uint64_t* ids, const uint32_t* lists, uint64_t n) {
    if (n == 0) return;
    DeviceGuard dg;
    const uint64_t chunk = chunk_rows(g->dp);
    std::vector<uint32_t> asg_store;
    const uint32_t* asg = lists;
    if (!asg) {
        asg_store.resize(n);
        vdb_ivf& m0 = *g->members[0];
        m0.set_device();
        DevBuf<float> dv, tmp;
        DevBuf<uint32_t> da;
        for (uint64_t r0 = 0; r0 < n; r0 += chunk) {
            const uint64_t c = std::min(chunk, n - r0);
            HIPCHECK(hipMemcpyAsync(dv.ensure(c * g->dim), v + r0 * g->dim, c * g->dim * 4, hipMemcpyHostToDevice,
                                    m0.stream));
            m0.assign(m0.padded_rows(dv.p, c, tmp), c, da.ensure(c));
            HIPCHECK(hipMemcpyAsync(asg_store.data() + r0, da.p, c * 4, hipMemcpyDeviceToHost, m0.stream));
            HIPCHECK(hipStreamSynchronize(m0.stream));
        }
        asg = asg_store.data();
    } else {
        for (uint64_t i = 0; i < n; ++i) require(asg[i] < g->nlist, "list id out of range");
    }
    place(g, asg, n);
    for_members(g, [&](size_t m) {
        for (uint64_t r0 = 0; r0 < n; r0 += chunk) {
            const uint64_t c = std::min(chunk, n - r0);
            g->members[m]->add_to_lists_host(v + r0 * g->dim, ids + r0, asg + r0, c);
        }
    });
    sync_counts(g);
}

// add / add_to_lists from rows on member 0's device: member 0 appends in place, the
// other members receive the rows by peer copies (xGMI), chunk by chunk.
void add_device(vdb_ivf* g, const float* d_v, const uint64_t* d_ids, const uint32_t* d_lists, uint64_t n) {
    if (n == 0) return;
    DeviceGuard dg;
    vdb_ivf& m0 = *g->members[0];
    m0.set_device();
    DevBuf<float> tmp;
    DevBuf<uint32_t> da;
    const float* vpad = m0.padded_rows(d_v, n, tmp);
    const uint32_t* dl = d_lists;
    if (!dl) {
        m0.assign(vpad, n, da.ensure(n));
        dl = da.p;
    }
    std::vector<uint32_t> h(n);
    HIPCHECK(hipMemcpyAsync(h.data(), dl, n * 4, hipMemcpyDeviceToHost, m0.stream));
    HIPCHECK(hipStreamSynchronize(m0.stream));
    for (uint64_t i = 0; i < n; ++i) require(h[i] < g->nlist, "list id out of range");
    place(g, h.data(), n);
    const uint64_t chunk = chunk_rows(g->dp);
    for_members(g, [&](size_t m) {
        vdb_ivf& mb = *g->members[m];
        if (m == 0 || mb.device == m0.device) {
            mb.append(vpad, d_ids, dl, n);
            return;
        }
        DevBuf<float> rv;
        DevBuf<uint64_t> ri;
        DevBuf<uint32_t> rl;
        for (uint64_t r0 = 0; r0 < n; r0 += chunk) {
            const uint64_t c = std::min(chunk, n - r0);
            HIPCHECK(hipMemcpyPeerAsync(rv.ensure(c * g->dp), mb.device, vpad + r0 * g->dp, m0.device,
                                        c * g->dp * 4, mb.stream));
            HIPCHECK(hipMemcpyPeerAsync(ri.ensure(c), mb.device, d_ids + r0, m0.device, c * 8, mb.stream));
            HIPCHECK(hipMemcpyPeerAsync(rl.ensure(c), mb.device, dl + r0, m0.device, c * 4, mb.stream));
            mb.append(rv.p, ri.p, rl.p, c);  // synchronises mb.stream before the buffers are reused
        }
    });
    sync_counts(g);
}

uint64_t gpu_bytes(const vdb_ivf* g, bool allocated) {
    uint64_t b = 0;
    for (auto& mb : g->members) b += allocated ? vdb_ivf_gpu_bytes_allocated(mb.get()) : vdb_ivf_gpu_bytes(mb.get());
    if (allocated) b += g->device_footprint();  // (the group's own host-API staging and stream buffers)
    return b;
}

void set_option(vdb_ivf* g, const std::string& name, int64_t value) {
    if (name == "coalesce") {
        g->coalesce = value != 0;
        return;
    }
    if (name == "coalesce_max_queries") {
        require(value > 0 && value < (1ll << 31), "coalesce_max_queries out of range");
        g->coalesce_max_queries = (uint32_t)value;
        return;
    }
    if (name == "coalesce_window_us") {
        require(value >= 0 && value < 1000000, "coalesce_window_us out of range");
        g->coalesce_window_us = (uint32_t)value;
        return;
    }
    DeviceGuard dg;
    for (auto& mb : g->members)
        if (vdb_ivf_set_option(mb.get(), name.c_str(), value) != VDB_OK) throw VdbError(VDB_ERR_INVALID_ARGUMENT, g_last_error);
    if (name == "batch") g->batch = (uint32_t)value;
    if (name == "stale_slots") g->stale = value ? 1 : 0;
    if (name == "coarse_mode") g->coarse_mode = (int)value;
}

void synchronize(vdb_ivf* g) {
    DeviceGuard dg;
    for (auto& mb : g->members) {
        mb->set_device();
        HIPCHECK(hipStreamSynchronize(mb->stream));
        for (auto& sl : mb->slots)
            if (sl.gstream) HIPCHECK(hipStreamSynchronize(sl.gstream));
    }
    g->set_device();
    HIPCHECK(hipStreamSynchronize(g->stream));
}

}  // namespace group
}  // namespace vdbe

// One search call over every member: the batch's queries go to every member (RCCL
// broadcast from member 0), each member runs the batch over its lists into its packed
// record, ONE all-gather per batch, member 0 merges into the caller's buffers. Member 0
// runs on the caller's stream; the others on their slot's stream, fenced by events
// against the caller's stream at both ends.
void vdb_ivf::group_search_device(const float* d_q, uint32_t n, uint32_t P, uint32_t k, float* d_dist,
                                  uint64_t* d_ids, hipStream_t s, const uint32_t* req_start) {
    DeviceGuard dg;
    const uint32_t M = (uint32_t)members.size();
    if (gev.empty()) {  // [0] caller -> members, [1 + m] member m's batch done, [1 + M] copies done,
                        // [2 + M + m] member m's call done (each created on its stream's device)
        gev.assign(2 * M + 2, nullptr);
        for (uint32_t e = 0; e < 2 * M + 2; ++e) {
            const uint32_t m = (e >= 1 && e <= M) ? e - 1 : (e >= M + 2 ? e - M - 2 : 0);
            HIPCHECK(hipSetDevice(members[m]->device));
            HIPCHECK(hipEventCreateWithFlags(&gev[e], hipEventDisableTiming));
        }
    }
    HIPCHECK(hipSetDevice(members[0]->device));
    HIPCHECK(hipEventRecord(gev[0], s));
    std::vector<SearchSlot*> w(M);
    std::vector<hipStream_t> ms(M);
    std::vector<const float*> qm(M, d_q);
    std::vector<const uint32_t*> rm(M, req_start);
    for (uint32_t m = 0; m < M; ++m) {
        vdb_ivf& mb = *members[m];
        mb.set_device();
        SearchSlot& peek = mb.slots[mb.next_slot];
        if (m > 0 && !peek.gstream) HIPCHECK(hipStreamCreateWithFlags(&peek.gstream, hipStreamNonBlocking));
        ms[m] = m == 0 ? s : peek.gstream;
        if (m > 0) HIPCHECK(hipStreamWaitEvent(ms[m], gev[0], 0));
        w[m] = &mb.begin_call(n, P, k, ms[m], M);
        if (m > 0) {
            qm[m] = mb.slot_buf(*w[m], w[m]->gq, (size_t)n * dim);
            if (req_start) rm[m] = mb.slot_buf(*w[m], w[m]->greq, n);
        }
    }
    // the queries (and request starts) onto every member
    if (M > 1) {
        if (group_rccl) {
            std::vector<hipStream_t> cs(M);
            for (uint32_t m = 0; m < M; ++m) {
                members[m]->set_device();
                cs[m] = members[m]->comm_enter(*w[m], ms[m]);
            }
            NCCLCHECK(ncclGroupStart());
            for (uint32_t m = 0; m < M; ++m) {
                NCCLCHECK(ncclBroadcast(d_q, (void*)qm[m], (size_t)n * dim, ncclFloat32, 0, members[m]->comm, cs[m]));
                if (req_start)
                    NCCLCHECK(ncclBroadcast(req_start, (void*)rm[m], n, ncclUint32, 0, members[m]->comm, cs[m]));
            }
            NCCLCHECK(ncclGroupEnd());
            for (uint32_t m = 0; m < M; ++m) {
                members[m]->set_device();
                members[m]->comm_leave(*w[m], ms[m]);
            }
        } else {  // members sharing one device (a rehearsal): plain device copies
            for (uint32_t m = 1; m < M; ++m) {
                members[m]->set_device();
                HIPCHECK(hipMemcpyAsync((void*)qm[m], d_q, (size_t)n * dim * 4, hipMemcpyDeviceToDevice, ms[m]));
                if (req_start)
                    HIPCHECK(hipMemcpyAsync((void*)rm[m], req_start, (size_t)n * 4, hipMemcpyDeviceToDevice, ms[m]));
            }
        }
    }
    // ONE exchange of every member's record of B queries, then member 0 merges them
    // into the caller's buffers (RCCL all-gather, or device copies on one device).
    auto exchange = [&](uint32_t B, float* od, uint64_t* oi) {
        const uint64_t rb = vdb_rank_record_bytes(B, k);
        if (group_rccl) {
            std::vector<hipStream_t> cs(M);
            for (uint32_t m = 0; m < M; ++m) {
                members[m]->set_device();
                cs[m] = members[m]->comm_enter(*w[m], ms[m]);
            }
            NCCLCHECK(ncclGroupStart());
            for (uint32_t m = 0; m < M; ++m)
                NCCLCHECK(ncclAllGather(w[m]->xrec.p, w[m]->xgat.p, rb, ncclUint8, members[m]->comm, cs[m]));
            NCCLCHECK(ncclGroupEnd());
            for (uint32_t m = 0; m < M; ++m) {
                members[m]->set_device();
                members[m]->comm_leave(*w[m], ms[m]);
            }
        } else {
            for (uint32_t m = 1; m < M; ++m) {
                members[m]->set_device();
                HIPCHECK(hipEventRecord(gev[1 + m], ms[m]));
            }
            members[0]->set_device();
            for (uint32_t m = 1; m < M; ++m) HIPCHECK(hipStreamWaitEvent(s, gev[1 + m], 0));
            for (uint32_t m = 0; m < M; ++m)
                HIPCHECK(hipMemcpyAsync(w[0]->xgat.p + (size_t)m * rb, w[m]->xrec.p, rb, hipMemcpyDeviceToDevice, s));
            HIPCHECK(hipEventRecord(gev[1 + M], s));  // members may overwrite their records after this
        }
        members[0]->set_device();
        merge_gathered(*w[0], M, B, k, od, oi, s);
    };
    if (group_tiered()) {
        // Members serving their lists through list caches (an index larger than HBM):
        // each member's tier cuts the call into sub-batches by what its own cache holds,
        // so every member writes the whole call's partials into one record (a member per
        // host thread: the tier plans loads and reads list files on the host), then ONE
        // exchange and one merge for the call.
        const uint64_t rb = vdb_rank_record_bytes(n, k);
        for (uint32_t m = 0; m < M; ++m) {
            members[m]->set_device();
            if (group_rccl || m == 0) members[m]->slot_buf(*w[m], w[m]->xgat, rb * M);
        }
        for_members(this, [&](size_t m) { members[m]->call_to_record(*w[m], qm[m], n, P, k, ms[m], rm[m]); });
        exchange(n, d_dist, d_ids);
    } else {
        uint32_t bmax = members[0]->batch_cap(P, k);  // (the smallest member cap: partial bytes per member)
        for (auto& mb : members) bmax = std::min(bmax, mb->batch_cap(P, k));
        for (uint32_t b0 = 0, B = std::min(bmax, n); b0 < n; b0 += B, B = std::min(B, n - b0)) {
            for (uint32_t m = 0; m < M; ++m) {
                vdb_ivf& mb = *members[m];
                mb.set_device();
                if (!group_rccl && m > 0 && b0 > 0) HIPCHECK(hipStreamWaitEvent(ms[m], gev[1 + M], 0));
                require(mb.run_batch(*w[m], qm[m] + (size_t)b0 * dim, B, P, k, rec_dist(*w[m]), rec_ids(*w[m], B, k),
                                     ms[m], rm[m], b0),
                        "group batch failed", VDB_ERR_STATE);
            }
            exchange(B, d_dist + (size_t)b0 * k, d_ids + (size_t)b0 * k);
        }
    }
    for (uint32_t m = 0; m < M; ++m) {
        vdb_ivf& mb = *members[m];
        mb.set_device();
        if (!group_rccl && m > 0) HIPCHECK(hipStreamWaitEvent(ms[m], gev[1 + M], 0));
        mb.end_call(*w[m], ms[m]);
        if (m > 0) HIPCHECK(hipEventRecord(gev[2 + M + m], ms[m]));
    }
    members[0]->set_device();
    for (uint32_t m = 1; m < M; ++m) HIPCHECK(hipStreamWaitEvent(s, gev[2 + M + m], 0));
}

extern "C" {

int vdb_ivf_create_group(const vdb_ivf_config* cfg, const int* devices, uint32_t ndev, vdb_ivf** out) {
    return guarded([&] {
        require(cfg && devices && out && ndev > 0, "null argument");
        require(ndev <= 64, "at most 64 devices per group", VDB_ERR_UNSUPPORTED);
        DeviceGuard dg;
        std::unique_ptr<vdb_ivf> g;
        {
            vdb_ivf_config c0 = *cfg;
            c0.device = devices[0];
            vdb_ivf* h = nullptr;
            if (vdb_ivf_create(&c0, &h) != VDB_OK) throw VdbError(VDB_ERR_DEVICE, g_last_error);
            g.reset(h);  // the group's own handle: host-API staging and stream on devices[0]
        }
        for (uint32_t m = 0; m < ndev; ++m) {
            vdb_ivf_config cm = *cfg;
            cm.device = devices[m];
            vdb_ivf* h = nullptr;
            if (vdb_ivf_create(&cm, &h) != VDB_OK) throw VdbError(VDB_ERR_DEVICE, g_last_error);
            g->members.emplace_back(h);
            h->rank = m;
            h->world = ndev;
            h->set_owned(std::vector<uint8_t>(cfg->nlist, 0));  // nothing placed yet
        }
        g->owner.assign(cfg->nlist, vdb_ivf::kUnplaced);
        g->owned.assign(cfg->nlist, 0);
        g->world = ndev;
        const std::set<int> distinct(devices, devices + ndev);
        g->group_rccl = distinct.size() == ndev;
        if (g->group_rccl) {
            for (uint32_t a = 0; a < ndev; ++a)
                for (uint32_t b = 0; b < ndev; ++b)
                    if (a != b) {
                        HIPCHECK(hipSetDevice(devices[a]));
                        (void)hipDeviceEnablePeerAccess(devices[b], 0);  // already enabled is fine
                        (void)hipGetLastError();
                    }
            std::vector<ncclComm_t> comms(ndev);
            NCCLCHECK(ncclCommInitAll(comms.data(), (int)ndev, devices));
            for (uint32_t m = 0; m < ndev; ++m) {
                g->members[m]->comm = comms[m];
                g->members[m]->comm_owned = true;
                g->members[m]->comm_rank = m;
                g->members[m]->comm_world = ndev;
                g->members[m]->set_device();
                g->members[m]->make_comm_stream();
            }
        }
        *out = g.release();
    });
}

uint32_t vdb_ivf_group_size(const vdb_ivf* h) { return h ? (h->is_group() ? (uint32_t)h->members.size() : 1u) : 0u; }

int vdb_ivf_list_owners(vdb_ivf* h, uint32_t* owner) {
    return guarded([&] {
        require(h && owner, "null argument");
        std::lock_guard<std::mutex> g(h->mu);
        for (uint32_t l = 0; l < h->nlist; ++l)
            owner[l] = h->is_group() ? h->owner[l] : (h->owned[l] ? h->rank : vdb_ivf::kUnplaced);
    });
}

int vdb_comm_unique_id(void* id) {
    return guarded([&] {
        require(id != nullptr, "null argument");
        ncclUniqueId u;
        NCCLCHECK(ncclGetUniqueId(&u));
        std::memcpy(id, &u, sizeof(u));
    });
}

int vdb_ivf_attach_comm(vdb_ivf* h, const void* id, uint32_t rank, uint32_t world) {
    return guarded([&] {
        require(h && id && world > 0 && rank < world, "invalid argument");
        require(!h->is_group(), "a group handle owns its communicators", VDB_ERR_STATE);
        std::lock_guard<std::mutex> g(h->mu);
        // (exchange_emulate_world: a shard's handle times its exchange on a communicator of
        // world 1, records of W ranks' size; diagnostics of one rank's timeline)
        const bool emulated = world == 1 && h->xchg_emulate > 1 && h->world == h->xchg_emulate;
        require((h->rank == rank && h->world == world) || emulated,
                "attach_comm after set_shard / plan_shard with the same (rank, world)", VDB_ERR_STATE);
        h->set_device();
        h->quiesce();
        h->stop_watch();  // a new communicator starts with a clean deadline record
        if (h->comm && h->comm_owned) (void)ncclCommDestroy(h->comm);
        h->comm = nullptr;
        h->comm_rank = rank;
        h->comm_world = world;
        ncclUniqueId u;
        std::memcpy(&u, id, sizeof(u));
        // Non-blocking init polled against comm_timeout_ms: a rank that never joins ends
        // in an error naming this rank (the communicator is aborted: no kernel has used
        // it yet) instead of a hang inside ncclCommInitRank.
        ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
        cfg.blocking = 0;
        ncclComm_t c = nullptr;
        const ncclResult_t r = ncclCommInitRankConfig(&c, (int)world, u, (int)rank, &cfg);
        h->comm = c;
        try {
            if (r != ncclSuccess && r != ncclInProgress)
                throw VdbError(VDB_ERR_DEVICE, h->rank_tag() + "ncclCommInitRankConfig: " + ncclGetErrorString(r));
            if (!c) throw VdbError(VDB_ERR_DEVICE, h->rank_tag() + "ncclCommInitRankConfig returned no communicator");
            h->nccl_settle(r, "communicator init (ncclCommInitRankConfig)");
            h->make_comm_stream();
            // Every rank must run the same collectives and hold a disjoint part of one index:
            // compare the settings that decide the collectives and the global list sizes,
            // and check that every non-empty list is stored by exactly one rank (one
            // all-gather, which also proves the communicator end to end).
            const uint32_t nw = (h->nlist + 63) / 64;
            const size_t words = 5 + nw;
            std::vector<uint64_t> mine(words, 0);
            uint64_t fnv = 1469598103934665603ull;  // FNV-1a of the global list sizes
            for (uint32_t l = 0; l < h->nlist; ++l) {
                fnv = (fnv ^ h->count[l]) * 1099511628211ull;
                if (h->owned[l] && h->count[l]) mine[5 + l / 64] |= 1ull << (l % 64);
            }
            mine[0] = ((uint64_t)h->dim << 32) | h->nlist;
            mine[1] = ((uint64_t)(uint32_t)h->metric << 32) | h->batch;
            mine[2] = (uint64_t)h->stale;  // (the tier may differ between ranks: exchanges are per call)
            mine[3] = fnv;
            mine[4] = h->total;
            DevBuf<uint64_t> dm, dall;
            HIPCHECK(hipMemcpyAsync(dm.ensure(words), mine.data(), words * 8, hipMemcpyHostToDevice, h->comm_stream));
            h->nccl_settle(ncclAllGather(dm.p, dall.ensure(words * world), words, ncclUint64, c, h->comm_stream),
                           "settings all-gather at attach");
            std::vector<uint64_t> all(words * (size_t)world);
            HIPCHECK(hipMemcpyAsync(all.data(), dall.p, all.size() * 8, hipMemcpyDeviceToHost, h->comm_stream));
            const auto t0 = std::chrono::steady_clock::now();
            for (;;) {  // the deadline holds for the first collective too
                const hipError_t q = hipStreamQuery(h->comm_stream);
                if (q == hipSuccess) break;
                if (q != hipErrorNotReady) HIPCHECK(q);
                const double ms =
                    std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
                if (ms > h->comm_timeout_ms)
                    throw VdbError(VDB_ERR_DEVICE, h->rank_tag() + "settings all-gather at attach not complete after " +
                                                       std::to_string((int)ms) + " ms (comm_timeout_ms)");
                std::this_thread::sleep_for(std::chrono::microseconds(200));
            }
            for (uint32_t q = 0; q < world; ++q)
                require(std::equal(mine.begin(), mine.begin() + 5, all.begin() + words * q),
                        h->rank_tag() + "rank " + std::to_string(q) +
                            " differs in dimension, nlist, metric, batch, stale_slots or list sizes",
                        VDB_ERR_STATE);
            for (uint32_t wd = 0; wd < nw; ++wd) {
                uint64_t any = 0, twice = 0;
                for (uint32_t q = 0; q < world; ++q) {
                    const uint64_t b = all[words * q + 5 + wd];
                    twice |= any & b;
                    any |= b;
                }
                if (emulated) break;  // (one shard of W: it holds only its own lists)
                uint64_t nonempty = 0;
                for (uint32_t l = wd * 64; l < std::min(h->nlist, (wd + 1) * 64); ++l)
                    if (h->count[l]) nonempty |= 1ull << (l % 64);
                require(!twice && any == nonempty,
                        h->rank_tag() + "the ranks' shards do not partition the lists (list " +
                            std::to_string(wd * 64 + __builtin_ctzll(twice ? twice : (any ^ nonempty))) +
                            (twice ? " stored by two ranks)" : " stored by no rank)"),
                        VDB_ERR_STATE);
            }
        } catch (...) {
            if (h->comm) (void)ncclCommAbort(h->comm);
            h->comm = nullptr;
            h->comm_rank = 0;
            h->comm_world = 1;
            throw;
        }
        h->comm_owned = true;
    });
}

int vdb_ivf_comm_status(vdb_ivf* h, uint64_t* exchanges_issued, uint64_t* exchanges_done) {
    return guarded([&] {
        require(h != nullptr, "null handle");
        uint64_t is = 0, dn = 0;
        std::string err;
        if (h->watch) {
            std::lock_guard<std::mutex> g(h->watch->m);
            is = h->watch->issued;
            dn = h->watch->completed;
            err = h->watch->error;
        }
        if (exchanges_issued) *exchanges_issued = is;
        if (exchanges_done) *exchanges_done = dn;
        if (!err.empty()) throw VdbError(VDB_ERR_DEVICE, err);
    });
}

int vdb_ivf_detach_comm(vdb_ivf* h) {
    return guarded([&] {
        require(h != nullptr, "null handle");
        require(!h->is_group(), "a group handle owns its communicators", VDB_ERR_STATE);
        std::lock_guard<std::mutex> g(h->mu);
        h->set_device();
        // After a missed deadline the communicator is aborted, not destroyed (destroy
        // would wait for the stalled exchange): detach only once no stream still holds
        // that exchange queued (or let the process exit instead).
        const bool failed = h->comm_failed();
        if (!failed) h->quiesce();
        h->stop_watch();
        if (h->comm && h->comm_owned) {
            if (failed) (void)ncclCommAbort(h->comm);
            else NCCLCHECK(ncclCommDestroy(h->comm));
        }
        h->comm = nullptr;
        h->comm_rank = 0;
        h->comm_world = 1;
    });
}

}  // extern "C"
