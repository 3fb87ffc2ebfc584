// rand_read_probe.cpp — the disk's random-read ceiling for the screened tier's survivor-row
// reads: a file of <GiB> written once, then random reads through the engine's own
// io_uring reader (csrc/uring.hpp) at queue depth <qd>, O_DIRECT, for each access shape the
// tier can issue:
//   4k        one 4 KiB page at a 4 KiB-aligned offset
//   8k        two pages (a 3,072-B row that straddles a page boundary)
//   row512    a 3,072-B row at a 512-B-aligned offset (rows on a 512-B pitch: exact reads)
//   row4k     the 4 KiB-aligned superset of a 3,072-B row at a random 4-B offset (round 5's reads)
//   row512s   the 512-B-aligned superset of a 3,072-B row at a random 4-B offset
// Prints one JSON line per shape: reads/s, GB/s delivered, useful row GB/s. The O_DIRECT
// alignment the file system accepts (512 or 4096) is probed first.
// usage: rand_read_probe <dir> [GiB=16] [qd=256] [seconds per shape=6]
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "../cuda-acceleratedvectordatabaseengine_amd/csrc/uring.hpp"

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
    const std::string dir = argc > 1 ? argv[1] : "/tmp";
    const uint64_t gib = argc > 2 ? std::strtoull(argv[2], nullptr, 10) : 16;
    const unsigned qd = argc > 3 ? (unsigned)std::atoi(argv[3]) : 256;
    const double secs = argc > 4 ? std::atof(argv[4]) : 6.0;
    const std::string path = dir + "/rand_read_probe.bin";
    const uint64_t size = gib << 30;
    {  // write the file (not sparse: real blocks)
        const size_t chunk = 64u << 20;
        void* buf = nullptr;
        if (posix_memalign(&buf, 4096, chunk)) return 1;
        std::memset(buf, 7, chunk);
        const int w = ::open(path.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
        if (w < 0) { std::perror("open"); return 1; }
        const double t0 = now();
        for (uint64_t o = 0; o < size; o += chunk)
            if (::write(w, buf, chunk) != (ssize_t)chunk) { std::perror("write"); return 1; }
        ::fsync(w);
        ::close(w);
        std::printf("{\"write_GBps\": %.3f, \"file_GiB\": %llu}\n", size / (now() - t0) / 1e9, (unsigned long long)gib);
        std::free(buf);
    }
    const int fd = ::open(path.c_str(), O_RDONLY | O_DIRECT);
    if (fd < 0) { std::perror("open O_DIRECT"); return 1; }
    char* bounce = nullptr;
    const size_t slot = 12288;
    if (posix_memalign((void**)&bounce, 4096, slot * qd)) return 1;
    // the O_DIRECT alignment the file system accepts
    int align = 4096;
    if (::pread(fd, bounce, 512, 512) == 512) align = 512;
    std::printf("{\"odirect_align\": %d}\n", align);
    vdbe::UringReader ur(qd);
    std::printf("{\"io_uring\": %s, \"qd\": %u}\n", ur.uring() ? "true" : "false", qd);
    struct Shape {
        const char* name;
        uint32_t row;   // useful bytes
        int kind;       // 0 fixed-size aligned read of `len`; 1 superset of a row at a 4-B offset, granule g
        uint32_t len_or_g;
    };
    std::vector<Shape> shapes = {{"4k", 4096, 0, 4096},      {"8k", 8192, 0, 8192},
                                 {"row512", 3072, 2, 512},  {"row4k", 3072, 1, 4096},
                                 {"row512s", 3072, 1, 512}};
    std::mt19937_64 rng(7);
    // two rounds, the second in reverse order: the rate of this pool's disks drifts within a run
    std::vector<Shape> order = shapes;
    order.insert(order.end(), shapes.rbegin(), shapes.rend());
    int round = 0;
    for (const Shape& sh : order) {
        const int rnd = round++ < (int)shapes.size() ? 1 : 2;
        if ((sh.kind == 2 || (sh.kind == 1 && sh.len_or_g == 512)) && align != 512) continue;
        uint64_t done = 0, bytes = 0, useful = 0, issued = 0;
        std::vector<unsigned> free_slots(qd);
        for (unsigned i = 0; i < qd; ++i) free_slots[i] = i;
        const double t0 = now();
        double t = t0;
        while (t - t0 < secs) {
            while (!free_slots.empty()) {
                uint64_t a0, len;
                if (sh.kind == 0) {
                    a0 = (rng() % (size / sh.len_or_g - 1)) * sh.len_or_g;
                    len = sh.len_or_g;
                } else if (sh.kind == 2) {
                    a0 = (rng() % ((size - 8192) / 512)) * 512;
                    len = sh.row;
                } else {
                    const uint64_t off = (rng() % ((size - 16384) / 4)) * 4;
                    const uint64_t g = sh.len_or_g;
                    a0 = off / g * g;
                    len = (off + sh.row + g - 1) / g * g - a0;
                }
                const unsigned b = free_slots.back();
                free_slots.pop_back();
                ur.read(fd, bounce + (size_t)b * slot, (uint32_t)len, a0, ((uint64_t)b << 32) | (uint32_t)len);
                ++issued;
            }
            for (const auto& d : ur.wait(1)) {
                if (d.result < 0) { std::fprintf(stderr, "read: %s\n", std::strerror((int)-d.result)); return 1; }
                free_slots.push_back((unsigned)(d.tag >> 32));
                bytes += (uint64_t)d.result;
                useful += sh.kind == 0 ? (uint64_t)d.result : sh.row;
                ++done;
            }
            t = now();
        }
        ur.drain();
        const double el = now() - t0;
        std::printf("{\"round\": %d, \"shape\": \"%s\", \"reads_per_s\": %.0f, \"GBps_read\": %.3f, \"GBps_useful\": %.3f, "
                    "\"bytes_per_read\": %.0f, \"seconds\": %.2f}\n",
                    rnd, sh.name, done / el, bytes / el / 1e9, useful / el / 1e9, done ? (double)bytes / done : 0.0, el);
        std::fflush(stdout);
    }
    ::close(fd);
    ::unlink(path.c_str());
    return 0;
}
