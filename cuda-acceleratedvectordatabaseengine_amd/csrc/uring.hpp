// uring.hpp — a minimal io_uring reader on raw syscalls (no liburing in this image).
//
// The list-cache tier's file home reads whole lists from an index file into page-locked
// staging buffers (the reference's IOUringPrefetcher / ListPrefetcher intent,
// engine/prefetcher.cpp:116-376, prefetcher.h:139-183). One ring per handle; reads are
// IORING_OP_READ submissions carrying a caller tag; completions are reaped in any order.
// When io_uring_setup is not permitted (a seccomp profile, an old kernel), the same
// interface falls back to synchronous pread, so callers never branch on it.
#pragma once

#include <linux/io_uring.h>
#include <sys/mman.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <atomic>
#include <cerrno>
#include <cstdint>
#include <cstring>
#include <deque>
#include <stdexcept>
#include <string>

namespace vdbe {

class UringReader {
public:
    struct Done {
        uint64_t tag;
        int64_t result;  // bytes read, or -errno
    };

    explicit UringReader(unsigned entries = 64) {
        io_uring_params p;
        std::memset(&p, 0, sizeof(p));
        fd_ = (int)::syscall(__NR_io_uring_setup, entries, &p);
        if (fd_ < 0) return;  // fallback: pread
        sq_bytes_ = p.sq_off.array + p.sq_entries * sizeof(unsigned);
        cq_bytes_ = p.cq_off.cqes + p.cq_entries * sizeof(io_uring_cqe);
        sq_ptr_ = ::mmap(nullptr, sq_bytes_, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_POPULATE, fd_, IORING_OFF_SQ_RING);
        cq_ptr_ = ::mmap(nullptr, cq_bytes_, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_POPULATE, fd_, IORING_OFF_CQ_RING);
        sqes_bytes_ = p.sq_entries * sizeof(io_uring_sqe);
        sqes_ = (io_uring_sqe*)::mmap(nullptr, sqes_bytes_, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_POPULATE, fd_,
                                      IORING_OFF_SQES);
        if (sq_ptr_ == MAP_FAILED || cq_ptr_ == MAP_FAILED || sqes_ == MAP_FAILED) {
            release();
            return;
        }
        char* sq = (char*)sq_ptr_;
        char* cq = (char*)cq_ptr_;
        sq_head_ = (unsigned*)(sq + p.sq_off.head);
        sq_tail_ = (unsigned*)(sq + p.sq_off.tail);
        sq_mask_ = *(unsigned*)(sq + p.sq_off.ring_mask);
        sq_array_ = (unsigned*)(sq + p.sq_off.array);
        cq_head_ = (unsigned*)(cq + p.cq_off.head);
        cq_tail_ = (unsigned*)(cq + p.cq_off.tail);
        cq_mask_ = *(unsigned*)(cq + p.cq_off.ring_mask);
        cqes_ = (io_uring_cqe*)(cq + p.cq_off.cqes);
        entries_ = p.sq_entries;
    }
    ~UringReader() { release(); }
    UringReader(const UringReader&) = delete;
    UringReader& operator=(const UringReader&) = delete;

    bool uring() const { return fd_ >= 0; }
    unsigned capacity() const { return uring() ? entries_ : 1u << 30; }
    unsigned in_flight() const { return inflight_; }

    // Queue one read of `len` bytes at `off` into `buf` (submitted by the next wait()).
    void read(int file, void* buf, uint32_t len, uint64_t off, uint64_t tag) {
        if (!uring()) {  // synchronous fallback: complete now, report at the next wait()
            int64_t got = 0;
            char* p = (char*)buf;
            while (got < (int64_t)len) {
                const ssize_t r = ::pread(file, p + got, len - got, (off_t)(off + got));
                if (r < 0 && errno == EINTR) continue;
                if (r <= 0) {
                    got = r < 0 ? -errno : got;
                    break;
                }
                got += r;
            }
            ready_.push_back({tag, got});
            return;
        }
        if (inflight_ + pending_ >= entries_) throw std::runtime_error("io_uring submission queue full");
        const unsigned tail = *sq_tail_;
        const unsigned idx = tail & sq_mask_;
        io_uring_sqe* e = &sqes_[idx];
        std::memset(e, 0, sizeof(*e));
        e->opcode = IORING_OP_READ;
        e->fd = file;
        e->addr = (uint64_t)(uintptr_t)buf;
        e->len = len;
        e->off = off;
        e->user_data = tag;
        sq_array_[idx] = idx;
        std::atomic_thread_fence(std::memory_order_release);
        *sq_tail_ = tail + 1;
        ++pending_;
    }

    // Submit queued reads and wait for at least `min_done` completions (0: just reap).
    std::deque<Done> wait(unsigned min_done) {
        std::deque<Done> out;
        if (!uring()) {
            out.swap(ready_);
            return out;
        }
        // io_uring_enter returns how many queued entries the kernel consumed; a partial
        // submission (or an EINTR after some were taken) leaves the rest queued, so submit
        // until none is pending. Completions already in the ring count toward `want`.
        const unsigned want = std::min(min_done, inflight_ + pending_);
        bool waited = want == 0;
        while (pending_ || !waited) {
            const unsigned submit = pending_;
            const int r = (int)::syscall(__NR_io_uring_enter, fd_, submit, want, want ? IORING_ENTER_GETEVENTS : 0u,
                                         nullptr, 0);
            if (r < 0) {
                if (errno == EINTR) continue;
                throw std::runtime_error(std::string("io_uring_enter: ") + std::strerror(errno));
            }
            if ((unsigned)r > submit) throw std::runtime_error("io_uring_enter consumed more entries than queued");
            if (r == 0 && submit) throw std::runtime_error("io_uring_enter consumed none of the queued reads");
            inflight_ += (unsigned)r;
            pending_ -= (unsigned)r;
            waited = true;  // a successful enter with GETEVENTS has waited for `want`
        }
        unsigned head = *cq_head_;
        std::atomic_thread_fence(std::memory_order_acquire);
        while (head != *cq_tail_) {
            const io_uring_cqe& c = cqes_[head & cq_mask_];
            out.push_back({c.user_data, (int64_t)c.res});
            ++head;
            --inflight_;
        }
        std::atomic_thread_fence(std::memory_order_release);
        *cq_head_ = head;
        return out;
    }

    // Forget every read: submit what is queued, wait for every read in flight and drop
    // the completions (after a failed load, so no stale completion reaches the next one).
    void drain() noexcept {
        try {
            while (pending_ || inflight_) (void)wait(inflight_ ? 1 : 0);
        } catch (...) {
            pending_ = inflight_ = 0;  // the ring is unusable; the owner discards the reader
        }
        ready_.clear();
    }

private:
    void release() {
        if (sqes_ && sqes_ != MAP_FAILED) ::munmap(sqes_, sqes_bytes_);
        if (cq_ptr_ && cq_ptr_ != MAP_FAILED) ::munmap(cq_ptr_, cq_bytes_);
        if (sq_ptr_ && sq_ptr_ != MAP_FAILED) ::munmap(sq_ptr_, sq_bytes_);
        sqes_ = nullptr;
        cq_ptr_ = sq_ptr_ = nullptr;
        if (fd_ >= 0) ::close(fd_);
        fd_ = -1;
    }

    int fd_ = -1;
    void* sq_ptr_ = nullptr;
    void* cq_ptr_ = nullptr;
    io_uring_sqe* sqes_ = nullptr;
    size_t sq_bytes_ = 0, cq_bytes_ = 0, sqes_bytes_ = 0;
    unsigned *sq_head_ = nullptr, *sq_tail_ = nullptr, *sq_array_ = nullptr;
    unsigned *cq_head_ = nullptr, *cq_tail_ = nullptr;
    unsigned sq_mask_ = 0, cq_mask_ = 0, entries_ = 0;
    io_uring_cqe* cqes_ = nullptr;
    unsigned inflight_ = 0, pending_ = 0;
    std::deque<Done> ready_;
};

}  // namespace vdbe
