// oracle/cpu_ref.cpp — TEST INFRASTRUCTURE ONLY (the parity checker, never the product).
//
// A CPU restatement of the reference's IVF-Flat CPU path: IVFFlatIndex with
// use_gpu=false in /root/reference/engine/ivf_flat_index.cpp. Every function cites
// the lines it restates. Arithmetic contract: fp32 throughout;
// L2 term = (a-b) rounded, squared rounded, added rounded (no FMA: built with
// -ffp-contract=off); sums run d = 0..D-1 from 0.0f; IP accumulates a*b then negates.
// Ordering contract: probes by (dist, list_id), candidates by (dist, id),
// merge dedupes by id keeping the first (smallest) occurrence, pads with
// FLT_MAX / UINT64_MAX.
//
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this.
#include "cpu_ref.h"

#include <algorithm>
#include <cfloat>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <random>
#include <unordered_set>
#include <utility>
#include <vector>
#ifdef _OPENMP
#include <omp.h>
#endif

namespace {

enum : int { kL2 = 0, kIP = 1, kCosine = 2 };

struct List {
    std::vector<float> vectors;  // row-major count x dim, add order (cpp:179-190)
    std::vector<uint64_t> ids;
    uint64_t count = 0;
};

using Cand = std::pair<float, uint64_t>;

// Distance exactly as the CPU branches compute it (cpp:308-318, 352-362, 275-285).
// Cosine has no CPU branch, so its distance stays 0.0f.
inline float distance(int metric, const float* a, const float* b, uint32_t dim) {
    float dist = 0.0f;
    if (metric == kL2) {
        for (uint32_t d = 0; d < dim; ++d) {
            float diff = a[d] - b[d];
            dist += diff * diff;
        }
    } else if (metric == kIP) {
        for (uint32_t d = 0; d < dim; ++d) dist += a[d] * b[d];
        dist = -dist;
    }
    return dist;
}

// k-means++ always measures plain L2 (cpp:77-81), whatever the index metric.
inline float l2(const float* a, const float* b, uint32_t dim) {
    float dist = 0.0f;
    for (uint32_t d = 0; d < dim; ++d) {
        float diff = a[d] - b[d];
        dist += diff * diff;
    }
    return dist;
}

}  // namespace

struct oracle_ivf {
    uint32_t dim;
    uint32_t nlist;
    int metric;
    std::vector<float> centroids;  // nlist x dim, zero-initialised (cpp:22)
    std::vector<List> lists;
    uint64_t total = 0;

    // assign_to_lists, cpp:259-295: strict '<' keeps the lowest centroid on ties.
    void assign(const float* v, uint64_t n, uint32_t* out) const {
        for (uint64_t i = 0; i < n; ++i) {
            const float* vec = v + i * dim;
            float best = std::numeric_limits<float>::max();
            uint32_t best_list = 0;
            for (uint32_t c = 0; c < nlist; ++c) {
                float dist = distance(metric, vec, centroids.data() + (size_t)c * dim, dim);
                if (dist < best) {
                    best = dist;
                    best_list = c;
                }
            }
            out[i] = best_list;
        }
    }

    // select_nprobe_lists, cpp:298-336.
    std::vector<uint32_t> select(const float* q, uint32_t nprobe) const {
        std::vector<std::pair<float, uint32_t>> cd;
        cd.reserve(nlist);
        for (uint32_t c = 0; c < nlist; ++c)
            cd.emplace_back(distance(metric, q, centroids.data() + (size_t)c * dim, dim), c);
        uint32_t take = std::min(nprobe, nlist);
        std::partial_sort(cd.begin(), cd.begin() + take, cd.end());
        std::vector<uint32_t> out(take);
        for (uint32_t p = 0; p < take; ++p) out[p] = cd[p].second;
        return out;
    }

    // search_list_cpu, cpp:339-384, with k already min(k, count) as search passes it.
    void scan_list(uint32_t l, const float* q, uint32_t k, std::vector<Cand>& out) const {
        const List& L = lists[l];
        if (L.ids.size() != L.count) {  // a count-only list (oracle_list_set_count) has no rows to scan
            std::fprintf(stderr, "oracle: list %u holds no rows (count-only)\n", l);
            std::abort();
        }
        std::vector<Cand> cand;
        cand.reserve(L.count);
        for (uint64_t i = 0; i < L.count; ++i)
            cand.emplace_back(distance(metric, q, L.vectors.data() + i * dim, dim), L.ids[i]);
        uint32_t take = std::min<uint64_t>(k, cand.size());
        std::partial_sort(cand.begin(), cand.begin() + take, cand.end());
        out.assign(cand.begin(), cand.begin() + take);
        // cpp:380-383 pads to k; search passes k == take, so nothing is padded.
    }
};

namespace {

// merge_results, cpp:474-518.
void merge(const std::vector<const std::vector<Cand>*>& slots, uint32_t k, float* D, uint64_t* I) {
    std::vector<Cand> all;
    for (const auto* s : slots)
        for (const Cand& c : *s)
            if (c.second != UINT64_MAX) all.push_back(c);
    std::sort(all.begin(), all.end());
    std::vector<Cand> uniq;
    std::unordered_set<uint64_t> seen;
    for (const Cand& c : all)
        if (seen.insert(c.second).second) uniq.push_back(c);
    uint32_t n = std::min<uint64_t>(k, uniq.size());
    for (uint32_t i = 0; i < n; ++i) {
        D[i] = uniq[i].first;
        I[i] = uniq[i].second;
    }
    for (uint32_t i = n; i < k; ++i) {
        D[i] = std::numeric_limits<float>::max();
        I[i] = UINT64_MAX;
    }
}

struct Slot {
    std::vector<Cand> res;
    int64_t source = -1;  // list whose scan filled this slot (-1: never filled)
};

// The per-query loop of IVFFlatIndex::search (cpp:205-256), with the slot vector
// allocated once per call (cpp:210-211) so an empty probed list leaves the previous
// query's slot content in place. `scan` yields slot results.
template <class ScanFn, class EmitFn>
void run_search(const oracle_ivf* h, const float* queries, uint32_t n, uint32_t nprobe,
                ScanFn&& scan, EmitFn&& emit) {
    uint32_t P = std::min(nprobe, h->nlist);  // clamp: cpp:218-222 is UB beyond nlist
    std::vector<Slot> slots(P);
    for (uint32_t q = 0; q < n; ++q) {
        const float* query = queries + (size_t)q * h->dim;
        std::vector<uint32_t> probes = h->select(query, nprobe);
        for (uint32_t p = 0; p < P; ++p) {
            uint32_t l = probes[p];
            if (h->lists[l].count == 0) continue;  // cpp:225
            scan(q, p, l, query, slots[p].res);
            slots[p].source = l;
        }
        emit(q, slots);
    }
}

}  // namespace

extern "C" {

oracle_ivf* oracle_create(uint32_t dim, uint32_t nlist, int metric) {
    if (dim == 0 || nlist == 0) return nullptr;  // cpp:17-19 throws invalid_argument
    oracle_ivf* h = new oracle_ivf();
    h->dim = dim;
    h->nlist = nlist;
    h->metric = metric;
    h->centroids.assign((size_t)nlist * dim, 0.0f);
    h->lists.resize(nlist);
    return h;
}

void oracle_destroy(oracle_ivf* h) { delete h; }

// k-means++ seeding of train, cpp:52-104.
void oracle_train_seed_only(oracle_ivf* h, const float* v, uint64_t n) {
    const uint32_t dim = h->dim;
    std::mt19937 gen(42);
    std::uniform_int_distribution<uint64_t> pick(0, n - 1);
    uint64_t first = pick(gen);
    std::memcpy(h->centroids.data(), v + first * dim, dim * sizeof(float));

    // k-means++ seeding, cpp:63-104.
    for (uint32_t c = 1; c < h->nlist; ++c) {
        std::vector<float> mind(n);
        float total = 0.0f;
        for (uint64_t i = 0; i < n; ++i) {
            float m = std::numeric_limits<float>::max();
            for (uint32_t e = 0; e < c; ++e)
                m = std::min(m, l2(v + i * dim, h->centroids.data() + (size_t)e * dim, dim));
            mind[i] = m;
            total += m;
        }
        std::uniform_real_distribution<float> prob(0.0f, total);
        float target = prob(gen);
        float cumsum = 0.0f;
        for (uint64_t i = 0; i < n; ++i) {
            cumsum += mind[i];
            if (cumsum >= target) {
                std::memcpy(h->centroids.data() + (size_t)c * dim, v + i * dim, dim * sizeof(float));
                break;
            }
        }
    }

}

// train, cpp:49-145: seeding then 10 Lloyd iterations (cpp:107-142).
void oracle_train(oracle_ivf* h, const float* v, uint64_t n) {
    const uint32_t dim = h->dim;
    oracle_train_seed_only(h, v, n);
    std::vector<uint32_t> asg(n);
    for (int it = 0; it < 10; ++it) {
        h->assign(v, n, asg.data());
        std::vector<std::vector<float>> sums(h->nlist, std::vector<float>(dim, 0.0f));
        std::vector<uint32_t> counts(h->nlist, 0);
        for (uint64_t i = 0; i < n; ++i) {
            uint32_t c = asg[i];
            for (uint32_t d = 0; d < dim; ++d) sums[c][d] += v[i * dim + d];
            counts[c]++;
        }
        for (uint32_t c = 0; c < h->nlist; ++c)
            if (counts[c] > 0)
                for (uint32_t d = 0; d < dim; ++d)
                    h->centroids[(size_t)c * dim + d] = sums[c][d] / counts[c];
    }
}

// add, cpp:148-202.
void oracle_add(oracle_ivf* h, const float* v, const uint64_t* ids, uint64_t n) {
    const uint32_t dim = h->dim;
    std::vector<uint32_t> asg(n);
    h->assign(v, n, asg.data());
    std::vector<std::vector<uint64_t>> members(h->nlist);
    for (uint64_t i = 0; i < n; ++i) members[asg[i]].push_back(i);
    for (uint32_t l = 0; l < h->nlist; ++l) {
        if (members[l].empty()) continue;
        List& L = h->lists[l];
        uint64_t old = L.count, now = old + members[l].size();
        L.vectors.resize(now * dim);
        L.ids.resize(now);
        for (size_t j = 0; j < members[l].size(); ++j) {
            uint64_t src = members[l][j];
            std::memcpy(L.vectors.data() + (old + j) * dim, v + src * dim, dim * sizeof(float));
            L.ids[old + j] = ids[src];
        }
        L.count = now;
    }
    h->total += n;
}

void oracle_search(oracle_ivf* h, const float* queries, uint32_t n, uint32_t nprobe, uint32_t k,
                   float* D, uint64_t* I) {
    run_search(
        h, queries, n, nprobe,
        [&](uint32_t, uint32_t, uint32_t l, const float* q, std::vector<Cand>& out) {
            h->scan_list(l, q, std::min<uint64_t>(k, h->lists[l].count), out);
        },
        [&](uint32_t q, const std::vector<Slot>& slots) {
            std::vector<const std::vector<Cand>*> ptrs;
            for (const Slot& s : slots) ptrs.push_back(&s.res);
            merge(ptrs, k, D + (size_t)q * k, I + (size_t)q * k);
        });
}

void oracle_search_mt(oracle_ivf* h, const float* queries, uint32_t n, uint32_t nprobe, uint32_t k,
                      float* D, uint64_t* I, int threads) {
    // Scans are independent per (query, probe); only the stale-slot carry is serial,
    // so scan in parallel first and replay the slot logic serially afterwards.
    uint32_t P = std::min(nprobe, h->nlist);
    std::vector<std::vector<Cand>> res((size_t)n * P);
#ifdef _OPENMP
    int nt = threads > 0 ? threads : omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 1) num_threads(nt)
#endif
    for (int64_t q = 0; q < (int64_t)n; ++q) {
        const float* query = queries + (size_t)q * h->dim;
        std::vector<uint32_t> probes = h->select(query, nprobe);
        for (uint32_t p = 0; p < P; ++p) {
            uint32_t l = probes[p];
            if (h->lists[l].count == 0) continue;
            h->scan_list(l, query, std::min<uint64_t>(k, h->lists[l].count), res[(size_t)q * P + p]);
        }
    }
    (void)threads;
    run_search(
        h, queries, n, nprobe,
        [&](uint32_t q, uint32_t p, uint32_t, const float*, std::vector<Cand>& out) {
            out = res[(size_t)q * P + p];
        },
        [&](uint32_t q, const std::vector<Slot>& slots) {
            std::vector<const std::vector<Cand>*> ptrs;
            for (const Slot& s : slots) ptrs.push_back(&s.res);
            merge(ptrs, k, D + (size_t)q * k, I + (size_t)q * k);
        });
}

void oracle_search_shard(oracle_ivf* h, const float* queries, uint32_t n, uint32_t nprobe,
                         uint32_t k, const uint8_t* owned, float* D, uint64_t* I) {
    static const std::vector<Cand> kEmpty;
    run_search(
        h, queries, n, nprobe,
        [&](uint32_t, uint32_t, uint32_t l, const float* q, std::vector<Cand>& out) {
            if (owned[l]) h->scan_list(l, q, std::min<uint64_t>(k, h->lists[l].count), out);
            else out.clear();
        },
        [&](uint32_t q, const std::vector<Slot>& slots) {
            std::vector<const std::vector<Cand>*> ptrs;
            for (const Slot& s : slots) ptrs.push_back(s.source >= 0 && owned[s.source] ? &s.res : &kEmpty);
            merge(ptrs, k, D + (size_t)q * k, I + (size_t)q * k);
        });
}

// oracle_search_shard with the scans of the (query, probe) pairs in parallel and the
// slot logic replayed serially afterwards (bit-identical to the serial version).
void oracle_search_shard_mt(oracle_ivf* h, const float* queries, uint32_t n, uint32_t nprobe, uint32_t k,
                            const uint8_t* owned, float* D, uint64_t* I, int threads) {
    static const std::vector<Cand> kEmpty;
    const uint32_t P = std::min(nprobe, h->nlist);
    std::vector<std::vector<uint32_t>> probes(n);
    for (uint32_t q = 0; q < n; ++q) probes[q] = h->select(queries + (size_t)q * h->dim, nprobe);
    std::vector<std::vector<Cand>> res((size_t)n * P);
#ifdef _OPENMP
    int nt = threads > 0 ? threads : omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 1) num_threads(nt)
#endif
    for (int64_t e = 0; e < (int64_t)n * P; ++e) {
        const uint32_t q = (uint32_t)(e / P), p = (uint32_t)(e % P);
        const uint32_t l = probes[q][p];
        if (!owned[l] || h->lists[l].count == 0) continue;
        h->scan_list(l, queries + (size_t)q * h->dim, std::min<uint64_t>(k, h->lists[l].count), res[e]);
    }
    (void)threads;
    run_search(
        h, queries, n, nprobe,
        [&](uint32_t q, uint32_t p, uint32_t, const float*, std::vector<Cand>& out) { out = res[(size_t)q * P + p]; },
        [&](uint32_t q, const std::vector<Slot>& slots) {
            std::vector<const std::vector<Cand>*> ptrs;
            for (const Slot& s : slots) ptrs.push_back(s.source >= 0 && owned[s.source] ? &s.res : &kEmpty);
            merge(ptrs, k, D + (size_t)q * k, I + (size_t)q * k);
        });
}

// oracle_search_shard_mt with the lists streamed in one at a time (a shard larger than the
// checker's memory): begin records the call's probes, scan takes the (query, probe) pairs of
// the one list currently holding rows, finish replays the slot logic. Bit-identical to
// oracle_search_shard when every owned probed list is scanned once.
struct oracle_stream {
    oracle_ivf* h;
    std::vector<float> queries;
    uint32_t n, nprobe, P, k;
    std::vector<std::vector<uint32_t>> probes;
    std::vector<std::vector<std::pair<uint32_t, uint32_t>>> pairs_of;  // per list: its (query, probe) pairs
    std::vector<std::vector<Cand>> res;
};

oracle_stream* oracle_stream_begin(oracle_ivf* h, const float* queries, uint32_t n, uint32_t nprobe, uint32_t k) {
    oracle_stream* st = new oracle_stream{h, std::vector<float>(queries, queries + (size_t)n * h->dim), n, nprobe,
                                          std::min(nprobe, h->nlist), k, {}, {}, {}};
    st->probes.resize(n);
    st->pairs_of.resize(h->nlist);
    st->res.resize((size_t)n * st->P);
    for (uint32_t q = 0; q < n; ++q) {
        st->probes[q] = h->select(queries + (size_t)q * h->dim, nprobe);
        for (uint32_t p = 0; p < st->P; ++p) st->pairs_of[st->probes[q][p]].emplace_back(q, p);
    }
    return st;
}

uint32_t oracle_stream_probed(const oracle_stream* st, uint32_t l) { return (uint32_t)st->pairs_of[l].size(); }

void oracle_stream_scan(oracle_stream* st, uint32_t l, int threads) {
    const auto& pq = st->pairs_of[l];
    const uint64_t cnt = st->h->lists[l].count;
    if (!cnt) return;
#ifdef _OPENMP
    int nt = threads > 0 ? threads : omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 1) num_threads(nt)
#endif
    for (int64_t e = 0; e < (int64_t)pq.size(); ++e) {
        const uint32_t q = pq[e].first, p = pq[e].second;
        st->h->scan_list(l, st->queries.data() + (size_t)q * st->h->dim, std::min<uint64_t>(st->k, cnt),
                         st->res[(size_t)q * st->P + p]);
    }
    (void)threads;
}

void oracle_stream_finish(oracle_stream* st, const uint8_t* owned, float* D, uint64_t* I) {
    static const std::vector<Cand> kEmpty;
    const uint32_t P = st->P, k = st->k;
    run_search(
        st->h, st->queries.data(), st->n, st->nprobe,
        [&](uint32_t q, uint32_t p, uint32_t, const float*, std::vector<Cand>& out) { out = st->res[(size_t)q * P + p]; },
        [&](uint32_t q, const std::vector<Slot>& slots) {
            std::vector<const std::vector<Cand>*> ptrs;
            for (const Slot& s : slots) ptrs.push_back(s.source >= 0 && owned[s.source] ? &s.res : &kEmpty);
            merge(ptrs, k, D + (size_t)q * k, I + (size_t)q * k);
        });
    delete st;
}

void oracle_merge_ranks(const float* dist, const uint64_t* ids, uint32_t nranks, uint32_t n,
                        uint32_t k, float* out_dist, uint64_t* out_ids) {
    for (uint32_t q = 0; q < n; ++q) {
        std::vector<std::vector<Cand>> parts(nranks);
        std::vector<const std::vector<Cand>*> ptrs;
        for (uint32_t r = 0; r < nranks; ++r) {
            for (uint32_t j = 0; j < k; ++j) {
                size_t o = ((size_t)r * n + q) * k + j;
                parts[r].emplace_back(dist[o], ids[o]);
            }
            ptrs.push_back(&parts[r]);
        }
        merge(ptrs, k, out_dist + (size_t)q * k, out_ids + (size_t)q * k);
    }
}

void oracle_select_nprobe(oracle_ivf* h, const float* query, uint32_t nprobe, uint32_t* out) {
    std::vector<uint32_t> p = h->select(query, nprobe);
    std::copy(p.begin(), p.end(), out);
}

void oracle_assign(oracle_ivf* h, const float* v, uint64_t n, uint32_t* out) { h->assign(v, n, out); }

// The same per-row argmin, rows spread over OpenMP threads: each row's loop is exactly the
// serial one (cpp:259-295), so the result is bit-identical per row (checked on CPU against
// oracle_assign in tests/test_oracle.py) and full-scale shapes finish in seconds.
void oracle_assign_mt(oracle_ivf* h, const float* v, uint64_t n, uint32_t* out, int threads) {
    const uint64_t chunk = 64;
#ifdef _OPENMP
    const int nt = threads > 0 ? threads : omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 1) num_threads(nt)
#else
    (void)threads;
#endif
    for (uint64_t c0 = 0; c0 < n; c0 += chunk)
        h->assign(v + c0 * h->dim, std::min<uint64_t>(chunk, n - c0), out + c0);
}

void oracle_get_centroids(oracle_ivf* h, float* out) {
    std::memcpy(out, h->centroids.data(), h->centroids.size() * sizeof(float));
}

void oracle_set_centroids(oracle_ivf* h, const float* c) {
    std::memcpy(h->centroids.data(), c, h->centroids.size() * sizeof(float));
}

uint64_t oracle_list_count(oracle_ivf* h, uint32_t l) { return h->lists[l].count; }

void oracle_get_list(oracle_ivf* h, uint32_t l, float* vectors, uint64_t* ids) {
    const List& L = h->lists[l];
    if (vectors) std::memcpy(vectors, L.vectors.data(), L.count * h->dim * sizeof(float));
    if (ids) std::memcpy(ids, L.ids.data(), L.count * sizeof(uint64_t));
}

void oracle_set_list(oracle_ivf* h, uint32_t l, const float* vectors, const uint64_t* ids,
                     uint64_t count) {
    float* v;
    uint64_t* i;
    oracle_list_resize(h, l, count, &v, &i);
    if (count) {
        std::memcpy(v, vectors, count * h->dim * sizeof(float));
        std::memcpy(i, ids, count * sizeof(uint64_t));
    }
}

void oracle_list_resize(oracle_ivf* h, uint32_t l, uint64_t count, float** vectors, uint64_t** ids) {
    List& L = h->lists[l];
    h->total = h->total - L.count + count;
    L.count = count;
    L.vectors.resize(count * h->dim);
    L.ids.resize(count);
    *vectors = L.vectors.data();
    *ids = L.ids.data();
}

void oracle_list_set_count(oracle_ivf* h, uint32_t l, uint64_t count) {
    // A list stored on another shard: only its emptiness is read (the empty-list skip,
    // cpp:225), so keep its count and no rows; oracle_search_shard never scans it.
    List& L = h->lists[l];
    h->total = h->total - L.count + count;
    L.count = count;
    std::vector<float>().swap(L.vectors);
    std::vector<uint64_t>().swap(L.ids);
}

uint64_t oracle_total_vectors(oracle_ivf* h) { return h->total; }

void oracle_gen_normal(uint32_t seed, uint64_t n, float* out) {
    std::mt19937 gen(seed);
    std::normal_distribution<float> dist(0.0f, 1.0f);
    for (uint64_t i = 0; i < n; ++i) out[i] = dist(gen);
}

}  // extern "C"
