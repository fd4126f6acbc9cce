// Host shared-memory collectives: a stand-in for RCCL when several ranks
// share ONE GPU (RCCL refuses duplicate devices in a communicator).  Used to
// rehearse the sharded step -- the same plans, kernels and collective call
// sites as the RCCL path -- on a single-GPU box (tests/test_gpu_multirank.py,
// SVGD_HOSTCOMM=<name>).  Not a performance path: every collective
// synchronises the stream and stages through host memory.
//
// Layout of the POSIX shm segment "/<name>": a header (arrival counter and
// generation for a sense-reversing barrier) followed by `world` slots of
// SLOT_BYTES each.
#include "hostcomm.h"

#include <atomic>
#include <cerrno>
#include <chrono>
#include <cstring>
#include <fcntl.h>
#include <string>
#include <sys/mman.h>
#include <sys/stat.h>
#include <thread>
#include <unistd.h>
#include <vector>

namespace svgd_amd {

namespace {
constexpr size_t HDR = 256;

struct Header {
    std::atomic<int> arrived;
    std::atomic<int> generation;
    std::atomic<int> ready; // set by rank 0 once the segment is initialised
};
} // namespace

struct HostComm {
    int world = 1, rank = 0;
    size_t slot = 0;
    std::string name;
    char *base = nullptr;
    size_t bytes = 0;
    std::vector<char> tmp;
    Header *hdr() { return reinterpret_cast<Header *>(base); }
    char *slot_ptr(int r) { return base + HDR + (size_t)r * slot; }

    // sense-reversing barrier over the shm header (bounded wait)
    int barrier()
    {
        Header *h = hdr();
        const int gen = h->generation.load(std::memory_order_acquire);
        if (h->arrived.fetch_add(1, std::memory_order_acq_rel) == world - 1) {
            h->arrived.store(0, std::memory_order_relaxed);
            h->generation.fetch_add(1, std::memory_order_acq_rel);
            return 0;
        }
        const auto t0 = std::chrono::steady_clock::now();
        while (h->generation.load(std::memory_order_acquire) == gen) {
            std::this_thread::yield();
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(120)) return -1;
        }
        return 0;
    }
};

int hostcomm_create(HostComm **out, const char *name, int world, int rank, size_t slot_bytes)
{
    HostComm *c = new HostComm();
    c->world = world;
    c->rank = rank;
    c->slot = (slot_bytes + 255) / 256 * 256;
    c->name = std::string("/") + name;
    c->bytes = HDR + c->slot * (size_t)world;
    int fd = -1;
    if (rank == 0) {
        shm_unlink(c->name.c_str());
        fd = shm_open(c->name.c_str(), O_CREAT | O_RDWR, 0600);
        if (fd >= 0 && ftruncate(fd, (off_t)c->bytes) != 0) {
            close(fd);
            fd = -1;
        }
    } else {
        const auto t0 = std::chrono::steady_clock::now();
        while ((fd = shm_open(c->name.c_str(), O_RDWR, 0600)) < 0) {
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(60)) break;
            std::this_thread::sleep_for(std::chrono::milliseconds(5));
        }
        // wait until rank 0 has sized it
        struct stat st;
        while (fd >= 0 && fstat(fd, &st) == 0 && (size_t)st.st_size < c->bytes)
            std::this_thread::sleep_for(std::chrono::milliseconds(5));
    }
    if (fd < 0) {
        delete c;
        return -1;
    }
    void *p = mmap(nullptr, c->bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (p == MAP_FAILED) {
        delete c;
        return -1;
    }
    c->base = static_cast<char *>(p);
    if (rank == 0) {
        new (c->hdr()) Header();
        c->hdr()->arrived.store(0);
        c->hdr()->generation.store(0);
        c->hdr()->ready.store(1, std::memory_order_release);
    } else {
        while (c->hdr()->ready.load(std::memory_order_acquire) != 1)
            std::this_thread::sleep_for(std::chrono::milliseconds(1));
    }
    *out = c;
    return c->barrier();
}

void hostcomm_destroy(HostComm *c)
{
    if (!c) return;
    c->barrier();
    munmap(c->base, c->bytes);
    if (c->rank == 0) shm_unlink(c->name.c_str());
    delete c;
}

// In-place all-gather of `count` bytes per rank: rank r's part at buf + r*count.
int hostcomm_allgather(HostComm *c, char *dbuf, size_t count, hipStream_t stream)
{
    if (count > c->slot) return -2;
    if (hipStreamSynchronize(stream) != hipSuccess) return -3;
    if (hipMemcpy(c->slot_ptr(c->rank), dbuf + (size_t)c->rank * count, count,
                  hipMemcpyDeviceToHost) != hipSuccess)
        return -3;
    if (c->barrier()) return -1;
    for (int r = 0; r < c->world; ++r)
        if (r != c->rank &&
            hipMemcpy(dbuf + (size_t)r * count, c->slot_ptr(r), count, hipMemcpyHostToDevice) !=
                hipSuccess)
            return -3;
    return c->barrier();
}

template <class T> static int allreduce_sum(HostComm *c, T *dbuf, size_t cnt, hipStream_t stream)
{
    const size_t bytes = cnt * sizeof(T);
    if (bytes > c->slot) return -2;
    if (hipStreamSynchronize(stream) != hipSuccess) return -3;
    if (hipMemcpy(c->slot_ptr(c->rank), dbuf, bytes, hipMemcpyDeviceToHost) != hipSuccess) return -3;
    if (c->barrier()) return -1;
    c->tmp.assign(bytes, 0);
    T *acc = reinterpret_cast<T *>(c->tmp.data());
    for (int r = 0; r < c->world; ++r) { // same order on every rank
        const T *v = reinterpret_cast<const T *>(c->slot_ptr(r));
        for (size_t i = 0; i < cnt; ++i) acc[i] += v[i];
    }
    if (hipMemcpy(dbuf, acc, bytes, hipMemcpyHostToDevice) != hipSuccess) return -3;
    return c->barrier();
}

// Grouped point-to-point exchange (ncclSend / ncclRecv of one group): rank r
// sends rows [send[2q], send[2q+1]) of dsend (w doubles per row; n rows) to
// each rank q, and receives from each rank q the rows [recv[3q], recv[3q+1])
// into drecv + recv[3q+2] * w.  Faithful to what a peer can see: the slot's
// data is NaN except the ranges this rank sends, every sender's ranges are
// published in its slot's header and a receiver whose expected range differs
// fails (-4); drecv is NaN-filled before the pieces land.  (own0, own1: the
// caller's rows, unused here: like ncclSend, the send buffer is left as it
// was -- the caller's finish writes only the particles its units touch, so
// rows between a range's pieces keep their zeros.)  Returns 0 on success.
int hostcomm_exchange_f64(HostComm *c, double *dsend, size_t n, size_t w, const int64_t *send,
                          double *drecv, size_t recv_rows, const int64_t *recv, int64_t own0, int64_t own1,
                          hipStream_t stream)
{
    const size_t hdr = (size_t)c->world * 2 * sizeof(int64_t), data = n * w * sizeof(double);
    if (hdr + data > c->slot) return -2;
    if (hipStreamSynchronize(stream) != hipSuccess) return -3;
    char *mine = c->slot_ptr(c->rank);
    std::memcpy(mine, send, hdr);
    double *md = reinterpret_cast<double *>(mine + hdr);
    std::memset(md, 0xff, data);
    for (int q = 0; q < c->world; ++q) {
        const int64_t a = send[2 * q], b = send[2 * q + 1];
        if (q != c->rank && b > a &&
            hipMemcpy(md + (size_t)a * w, dsend + (size_t)a * w, (size_t)(b - a) * w * sizeof(double),
                      hipMemcpyDeviceToHost) != hipSuccess)
            return -3;
    }
    if (c->barrier()) return -1;
    int rc = 0;
    // (stream-ordered fills: a plain hipMemset may still run when the
    // stream's next kernel starts)
    if (recv_rows && (hipMemsetAsync(drecv, 0xff, recv_rows * w * sizeof(double), stream) != hipSuccess ||
                      hipStreamSynchronize(stream) != hipSuccess))
        rc = -3;
    for (int q = 0; q < c->world && !rc; ++q) {
        const int64_t a = recv[3 * q], b = recv[3 * q + 1], off = recv[3 * q + 2];
        if (q == c->rank) continue;
        const int64_t *ph = reinterpret_cast<const int64_t *>(c->slot_ptr(q));
        const int64_t pa = ph[2 * c->rank], pb = ph[2 * c->rank + 1];
        const bool sent = pb > pa, expected = b > a;
        if (sent != expected || (sent && (pa != a || pb != b))) {
            rc = -4; // the sender's range for this rank is not the one expected
            break;
        }
        if (b > a) {
            const double *src = reinterpret_cast<const double *>(c->slot_ptr(q) + hdr) + (size_t)a * w;
            if (hipMemcpy(drecv + (size_t)off * w, src, (size_t)(b - a) * w * sizeof(double),
                          hipMemcpyHostToDevice) != hipSuccess)
                rc = -3;
        }
    }
    const int brc = c->barrier();
    return rc ? rc : brc;
}

int hostcomm_allreduce_u32(HostComm *c, uint32_t *dbuf, size_t cnt, hipStream_t stream)
{
    return allreduce_sum(c, dbuf, cnt, stream);
}

int hostcomm_allreduce_f64(HostComm *c, double *dbuf, size_t cnt, hipStream_t stream)
{
    return allreduce_sum(c, dbuf, cnt, stream);
}

int hostcomm_allreduce_u64(HostComm *c, unsigned long long *dbuf, size_t cnt, hipStream_t stream)
{
    return allreduce_sum(c, dbuf, cnt, stream);
}

} // namespace svgd_amd
