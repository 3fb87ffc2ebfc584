// floor.hpp — the run-time floor under the screened scan: host logic only (no HIP), so the
// CPU tests drive it on synthetic reports (tests/cpp/floor_test.cpp).
//
// Every screened batch (lists in HBM) writes one report into a ring of page-locked host
// memory (ivf_screen_offsets, screen.hip): {survivors, or ~0 when its candidate buffer
// overflowed; its (query, vector) pairs; its sequence number; k x its valid (query, list)
// pairs (the survivors no screen can avoid)}. The device writes the three counts, then a
// system-scope release fence, then the sequence number; the host reads the sequence, the
// counts and the sequence again and takes the report only when both reads name the batch
// it expects, so a report can never pair one batch's sequence with another's counts.
//
// When a completed batch of at least `min_pairs` pairs overflowed, or its survivors beyond
// k per valid pair exceed `ppm` of its pairs (a data regime where the bound is wider than
// the distance spread: the exact re-checks then cost more than the exact scan saves), the
// next `skip` batches run the exact scan, twice as many after each further trip in a row
// (at most 32x); then the screen is retried on ONE batch (the probe), the batches issued
// while its report is outstanding running the exact scan. Reports are read in sequence
// order; the reports of batches already in flight at a trip belong to that trip. Results
// are the same either way; only speed changes.
#pragma once
#include <stdint.h>

#include <algorithm>
#include <atomic>

namespace vdbe {

struct ScreenFloor {
    static constexpr uint32_t kRing = 64;  // report entries (uint32 x 4 each), indexed by seq % kRing
    // probe reports still missing after this many batches planned meanwhile are given up
    // (a batch that never ran): the screen is retried rather than skipped for good
    static constexpr uint32_t kProbeWait = 256;

    uint32_t ppm = 50000;           // option screen_floor_ppm (0: never fall back)
    uint32_t skip = 32;             // option screen_floor_skip
    uint64_t min_pairs = 1u << 22;  // option screen_floor_min

    uint32_t seq = 0;         // the last sequence number issued to a screened batch
    uint32_t seen = 0;        // every report up to this sequence has been read (or given up)
    uint32_t skip_left = 0;   // exact batches still owed to the last trip
    uint32_t streak = 0;      // trips in a row (the backoff exponent)
    uint32_t probe = 0;       // the retry batch's sequence while its report is outstanding
    uint32_t probe_wait = 0;  // batches planned while it is outstanding
    uint32_t trip_seq = 0;    // the sequence issued last when the floor tripped
    uint64_t batches = 0;     // batches sent to the exact scan by the floor
    uint64_t trips = 0;
    uint64_t torn = 0;        // reports read while being written (retried at the next poll)
    uint64_t lost = 0;        // reports overwritten before they were read

    void reset_state() { skip_left = streak = probe = probe_wait = 0; }

    // One report entry of the ring, read so that it cannot tear: false while the entry
    // does not (yet) hold a consistent report of sequence number s.
    static bool read(const volatile uint32_t* e, uint32_t s, uint32_t out[4], bool* newer) {
        const uint32_t z1 = e[2];
        std::atomic_thread_fence(std::memory_order_acquire);
        out[0] = e[0];
        out[1] = e[1];
        out[3] = e[3];
        std::atomic_thread_fence(std::memory_order_acquire);
        const uint32_t z2 = e[2];
        out[2] = z2;
        *newer = z2 && (int32_t)(z2 - s) > 0;
        return z1 == s && z2 == s;
    }

    // Read every report that has arrived, in sequence order (stops at the first batch still
    // running), and apply the trip rule to each.
    template <class Ring>
    void poll(const Ring& ring) {
        while ((int32_t)(seq - seen) > 0) {
            const uint32_t s = seen + 1;
            if (s == 0) {  // (0 is never issued)
                seen = s;
                continue;
            }
            if (seq - s >= kRing) {  // the ring has wrapped past it: that report is gone
                ++lost;
                give_up(s);
                continue;
            }
            uint32_t v[4];
            bool newer = false;
            if (!read(ring(s % kRing), s, v, &newer)) {
                if (newer) {  // overwritten by a later batch's report
                    ++lost;
                    give_up(s);
                    continue;
                }
                // (not written yet, or being written: a later poll reads it)
                const uint32_t z = ring(s % kRing)[2];
                if (z == s) ++torn;
                return;
            }
            seen = s;
            apply(v);
        }
    }

    void give_up(uint32_t s) {
        seen = s;
        if (probe == s) probe = 0;  // (its verdict never comes: retry the screen later)
    }

    void apply(const uint32_t v[4]) {
        const uint32_t s = v[2];
        const bool was_probe = probe && s == probe;
        if (was_probe) probe = 0;
        if (!ppm || v[1] < min_pairs) return;
        if (trips && (int32_t)(s - trip_seq) <= 0) return;  // (in flight at the trip)
        const uint64_t excess = v[0] > v[3] ? (uint64_t)v[0] - v[3] : 0;
        if (v[0] == ~0u || excess * 1000000ull > (uint64_t)ppm * v[1]) {
            skip_left = skip << std::min<uint32_t>(streak, 5);
            ++streak;
            ++trips;
            trip_seq = seq;
        } else if (was_probe) {
            streak = 0;
        }
    }

    // Planning a batch the screen would serve: false sends it to the exact scan; true
    // returns, in *issue, the sequence number its report must carry.
    template <class Ring>
    bool plan(const Ring& ring, uint32_t* issue) {
        poll(ring);
        if (probe && ++probe_wait > kProbeWait) {
            probe_wait = 0;
            seen = std::max<uint32_t>(seen, probe);  // (every report up to it read or given up)
            probe = 0;
        }
        if (skip_left || probe) {
            if (skip_left) --skip_left;
            ++batches;
            return false;
        }
        const bool retry = streak > 0;
        if (!++seq) ++seq;  // (0: never written)
        *issue = seq;
        if (retry) {
            probe = seq;
            probe_wait = 0;
        }
        return true;
    }
};

}  // namespace vdbe
