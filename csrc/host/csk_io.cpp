// Native checkpoint reader (host side of the weight-distribution path,
// SURVEY §2.7 "Recommended weight-distribution scheme").
//
// The reference re-reads every model with `from_pretrained` on every job
// (swarm/diffusion/diffusion_func.py:41-46).  Here a model is read once per
// process (or 1/N of it per rank of a node, parallel/sharded.py) and this file
// is the part that moves the bytes: a byte range of a file goes
//
//   page cache --pread (T reader threads, one 16 MiB chunk each)--> pinned
//   staging slot (ring of 8, hipHostMalloc'd once per process)
//   --hipMemcpyAsync on the caller's stream--> device buffer
//
// so the reads of chunks i+1 .. i+6 overlap the H2D copy of chunk i and the
// PCIe link sees back-to-back pinned DMA (no pageable bounce buffer, no
// per-tensor open/seek/bytearray).  A host destination is filled by the
// readers directly (parallel pread, no staging).
//
// Protocol: chunk c uses slot c % NSLOT.  A reader may fill slot s for chunk c
// once free_for[s] == c (the copy of chunk c - NSLOT has completed); the copy
// thread (the caller) waits for ready[s] == c, issues the copy, records the
// slot's event and releases slots whose copies are done, keeping at most
// MAX_INFLIGHT copies queued.  Every wait is on a condition variable; a read
// error stops the readers and is returned after the queued copies drain.
#include <hip/hip_runtime_api.h>

#include <fcntl.h>
#include <unistd.h>

#include <atomic>
#include <cerrno>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <mutex>
#include <thread>
#include <vector>

#define CSKIO_API extern "C" __attribute__((visibility("default")))

namespace {

constexpr int NSLOT = 8;
constexpr long long SLOT_BYTES = 16ll << 20;
constexpr int MAX_INFLIGHT = 2;

struct Ring {
  char* buf[NSLOT] = {};
  hipEvent_t ev[NSLOT] = {};
  bool ok = false;
};

Ring g_ring;
std::mutex g_ring_mu;  // one transfer at a time owns the ring

int ring_init() {
  if (g_ring.ok) return 0;
  for (int s = 0; s < NSLOT; ++s) {
    hipError_t e = hipHostMalloc((void**)&g_ring.buf[s], SLOT_BYTES, hipHostMallocDefault);
    if (e != hipSuccess) return (int)e;
    e = hipEventCreateWithFlags(&g_ring.ev[s], hipEventDisableTiming);
    if (e != hipSuccess) return (int)e;
  }
  g_ring.ok = true;
  return 0;
}

// pread exactly n bytes (short reads continue; EOF before n is an error)
int pread_all(int fd, char* dst, long long n, long long off) {
  while (n > 0) {
    const ssize_t r = ::pread(fd, dst, (size_t)(n > (1ll << 30) ? (1ll << 30) : n), (off_t)off);
    if (r < 0) {
      if (errno == EINTR) continue;
      return -errno;
    }
    if (r == 0) return -EIO;  // file shorter than its header says
    dst += r;
    off += r;
    n -= r;
  }
  return 0;
}

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

}  // namespace

// Read [offset, offset + nbytes) of `path` into `dst`.
//   dst_is_device = 0: host memory, filled by `nthreads` parallel preads;
//   dst_is_device = 1: device memory, through the pinned ring on `stream`
//                      (returns after every copy has completed).
// stats (optional, 3 doubles): [0] seconds the readers spent in pread (sum over
// threads), [1] wall seconds of the whole call, [2] bytes moved.
// Returns 0, a negative errno (I/O) or a positive hipError_t.
CSKIO_API int csk_io_read(const char* path, long long offset, long long nbytes, void* dst, int dst_is_device,
                          int nthreads, hipStream_t stream, double* stats) {
  const double t_start = now_s();
  if (nbytes < 0 || offset < 0 || (!dst && nbytes > 0)) return -EINVAL;
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 32) nthreads = 32;
  const int fd = ::open(path, O_RDONLY | O_CLOEXEC);
  if (fd < 0) return -errno;
  const long long nchunks = (nbytes + SLOT_BYTES - 1) / SLOT_BYTES;
  std::atomic<long long> next{0};
  std::atomic<int> err{0};
  std::vector<double> busy(nthreads, 0.0);

  if (!dst_is_device) {
    std::vector<std::thread> th;
    for (int t = 0; t < nthreads; ++t)
      th.emplace_back([&, t]() {
        for (;;) {
          const long long c = next.fetch_add(1);
          if (c >= nchunks || err.load()) break;
          const long long o = c * SLOT_BYTES, n = std::min(SLOT_BYTES, nbytes - o);
          const double t0 = now_s();
          const int rc = pread_all(fd, (char*)dst + o, n, offset + o);
          busy[t] += now_s() - t0;
          if (rc) err.store(rc);
        }
      });
    for (auto& x : th) x.join();
    ::close(fd);
    if (stats) {
      double b = 0;
      for (double x : busy) b += x;
      stats[0] = b;
      stats[1] = now_s() - t_start;
      stats[2] = (double)nbytes;
    }
    return err.load();
  }

  std::lock_guard<std::mutex> own(g_ring_mu);
  int rc = ring_init();
  if (rc) {
    ::close(fd);
    return rc;
  }
  std::mutex mu;
  std::condition_variable cv;
  long long free_for[NSLOT], ready[NSLOT];
  for (int s = 0; s < NSLOT; ++s) {
    free_for[s] = s;  // slot s may take chunk s first
    ready[s] = -1;
  }
  bool stop = false;
  const int readers = std::min<long long>(nthreads, std::max<long long>(1, nchunks));
  std::vector<std::thread> th;
  for (int t = 0; t < readers; ++t)
    th.emplace_back([&, t]() {
      for (;;) {
        const long long c = next.fetch_add(1);
        if (c >= nchunks) break;
        const int s = (int)(c % NSLOT);
        {
          std::unique_lock<std::mutex> lk(mu);
          cv.wait(lk, [&] { return stop || free_for[s] == c; });
          if (stop) break;
        }
        const long long o = c * SLOT_BYTES, n = std::min(SLOT_BYTES, nbytes - o);
        const double t0 = now_s();
        const int r = pread_all(fd, g_ring.buf[s], n, offset + o);
        busy[t] += now_s() - t0;
        std::lock_guard<std::mutex> lk(mu);
        if (r) {
          if (!err.load()) err.store(r);
          stop = true;
        } else {
          ready[s] = c;
        }
        cv.notify_all();
        if (r) break;
      }
    });

  std::deque<long long> inflight;
  auto release_oldest = [&]() -> int {
    const long long j = inflight.front();
    inflight.pop_front();
    const int s = (int)(j % NSLOT);
    const hipError_t e = hipEventSynchronize(g_ring.ev[s]);
    std::lock_guard<std::mutex> lk(mu);
    free_for[s] = j + NSLOT;
    cv.notify_all();
    return (int)e;
  };
  for (long long c = 0; c < nchunks && !rc; ++c) {
    const int s = (int)(c % NSLOT);
    {
      std::unique_lock<std::mutex> lk(mu);
      cv.wait(lk, [&] { return stop || ready[s] == c; });
      if (stop) break;
    }
    const long long o = c * SLOT_BYTES, n = std::min(SLOT_BYTES, nbytes - o);
    hipError_t e = hipMemcpyAsync((char*)dst + o, g_ring.buf[s], (size_t)n, hipMemcpyHostToDevice, stream);
    if (e == hipSuccess) e = hipEventRecord(g_ring.ev[s], stream);
    if (e != hipSuccess) {
      rc = (int)e;
      break;
    }
    inflight.push_back(c);
    while ((int)inflight.size() > MAX_INFLIGHT && !rc) rc = release_oldest();
  }
  while (!inflight.empty()) {
    const int e = release_oldest();
    if (!rc) rc = e;
  }
  {
    std::lock_guard<std::mutex> lk(mu);
    stop = true;
    cv.notify_all();
  }
  for (auto& x : th) x.join();
  ::close(fd);
  if (stats) {
    double b = 0;
    for (double x : busy) b += x;
    stats[0] = b;
    stats[1] = now_s() - t_start;
    stats[2] = (double)nbytes;
  }
  if (err.load()) return err.load();
  return rc;
}

// Bytes of pinned staging the device path holds once used (for reports).
CSKIO_API long long csk_io_staging_bytes() { return g_ring.ok ? (long long)NSLOT * SLOT_BYTES : 0; }

// Free the pinned ring (tests; a worker keeps it for its lifetime).
CSKIO_API int csk_io_release() {
  std::lock_guard<std::mutex> own(g_ring_mu);
  if (!g_ring.ok) return 0;
  for (int s = 0; s < NSLOT; ++s) {
    (void)hipEventDestroy(g_ring.ev[s]);
    (void)hipHostFree(g_ring.buf[s]);
    g_ring.buf[s] = nullptr;
  }
  g_ring.ok = false;
  return 0;
}
