/* Probe (diagnostic): io_uring availability (raw syscalls), O_DIRECT support and
 * sequential read bandwidth of a file, buffered vs O_DIRECT. usage: io_probe <dir> <GiB> */
#define _GNU_SOURCE
#include <fcntl.h>
#include <linux/io_uring.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>
#include <errno.h>
static double now(void) { struct timespec t; clock_gettime(CLOCK_MONOTONIC, &t); return t.tv_sec + t.tv_nsec * 1e-9; }
int main(int argc, char** argv) {
    const char* dir = argc > 1 ? argv[1] : "/tmp";
    size_t gib = argc > 2 ? (size_t)atol(argv[2]) : 4;
    struct io_uring_params p; memset(&p, 0, sizeof(p));
    int fd = (int)syscall(__NR_io_uring_setup, 64, &p);
    printf("io_uring_setup: %s (errno %d)\n", fd >= 0 ? "ok" : "FAILED", fd >= 0 ? 0 : errno);
    if (fd >= 0) close(fd);
    char path[4096]; snprintf(path, sizeof(path), "%s/io_probe.bin", dir);
    size_t chunk = 64 << 20, total = gib << 30;
    void* buf; if (posix_memalign(&buf, 4096, chunk)) return 1;
    memset(buf, 7, chunk);
    int w = open(path, O_WRONLY | O_CREAT | O_TRUNC, 0644);
    if (w < 0) { perror("open w"); return 1; }
    double t0 = now();
    for (size_t o = 0; o < total; o += chunk) if (write(w, buf, chunk) != (ssize_t)chunk) { perror("write"); return 1; }
    fsync(w); close(w);
    printf("write %zu GiB: %.2f GB/s\n", gib, total / (now() - t0) / 1e9);
    int d = open(path, O_RDONLY | O_DIRECT);
    printf("O_DIRECT open: %s\n", d >= 0 ? "ok" : "FAILED");
    if (d >= 0) {
        t0 = now(); size_t got = 0; ssize_t r;
        while ((r = pread(d, buf, chunk, got)) > 0) got += r;
        printf("O_DIRECT pread %zu B: %.2f GB/s (%s)\n", got, got / (now() - t0) / 1e9, r < 0 ? strerror(errno) : "eof");
        close(d);
    }
    int b = open(path, O_RDONLY);
    t0 = now(); size_t got = 0; ssize_t r;
    while ((r = pread(b, buf, chunk, got)) > 0) got += r;
    printf("buffered pread (page cache likely warm): %.2f GB/s\n", got / (now() - t0) / 1e9);
    close(b);
    unlink(path);
    return 0;
}
