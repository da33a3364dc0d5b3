// Infinity Cache (MALL, 256 MiB) behaviour for a ring of intermediates:
//  write : 1 GiB of 16-B stores into a ring of R bytes (R = 1 GiB: no reuse)
//  read  : 1 GiB of 16-B loads from a ring of R bytes
//  rw    : item i writes ring slot i and reads slot i - lag (a producer and a
//          consumer of the same ring in one grid, lag slots apart)
// If dirty ring lines that are overwritten never reach HBM, 'write' at small
// R runs faster than HBM's write rate; 'read' at small R shows MALL read
// bandwidth.  One launch per measurement (no chunk launch tails).
//   hipcc --offload-arch=gfx950 -O3 tools/mall_probe.hip -o tools/mall_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                     \
  do {                                                            \
    hipError_t e = (x);                                           \
    if (e != hipSuccess) {                                        \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); \
      std::exit(1);                                               \
    }                                                             \
  } while (0)

// item = 64 KiB (4096 x 16 B), one 256-thread workgroup per item, 16 stores per thread
constexpr long ITEM = 4096;  // double2 per item

__global__ __launch_bounds__(256) void k_write(double2* ring, long ring_items, long items) {
  for (long it = blockIdx.x; it < items; it += gridDim.x) {
    double2* p = ring + (it % ring_items) * ITEM;
#pragma unroll
    for (int s = 0; s < 16; ++s) p[s * 256 + threadIdx.x] = make_double2((double)it, (double)s);
  }
}

__global__ __launch_bounds__(256) void k_read(const double2* ring, long ring_items, long items, double2* sink) {
  double2 acc = make_double2(0, 0);
  for (long it = blockIdx.x; it < items; it += gridDim.x) {
    const double2* p = ring + (it % ring_items) * ITEM;
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const double2 v = p[s * 256 + threadIdx.x];
      acc.x += v.x;
      acc.y += v.y;
    }
  }
  if (acc.x == 1.2345) sink[threadIdx.x] = acc;
}

// producer/consumer in one grid: item it writes slot it and reads slot it - lag
// (the read item was written lag items earlier in dispatch order)
__global__ __launch_bounds__(256) void k_rw(double2* ring, long ring_items, long items, long lag, double2* sink) {
  double2 acc = make_double2(0, 0);
  for (long it = blockIdx.x; it < items; it += gridDim.x) {
    double2* p = ring + (it % ring_items) * ITEM;
#pragma unroll
    for (int s = 0; s < 16; ++s) p[s * 256 + threadIdx.x] = make_double2((double)it, (double)s);
    if (it >= lag) {
      const double2* q = ring + ((it - lag) % ring_items) * ITEM;
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        const double2 v = q[s * 256 + threadIdx.x];
        acc.x += v.x;
        acc.y += v.y;
      }
    }
  }
  if (acc.x == 1.2345) sink[threadIdx.x] = acc;
}

// one 4-B load per `stride` bytes (translation warm-up, almost no data)
__global__ __launch_bounds__(256) void k_touch(const double2* base, long bytes, long stride, double2* sink) {
  double acc = 0;
  for (long o = ((long)blockIdx.x * 256 + threadIdx.x) * stride; o < bytes; o += (long)gridDim.x * 256 * stride)
    acc += reinterpret_cast<const double*>(reinterpret_cast<const char*>(base) + o)[0];
  if (acc == 1.2345) sink[0] = make_double2(acc, 0);
}

int main(int argc, char** argv) {
  const long total = 1L << 30;  // bytes per measurement
  const long items = total / (ITEM * 16);
  const long alloc = 4L << 30;
  double2 *ring, *sink;
  CK(hipMalloc(&ring, alloc));
  CK(hipMalloc(&sink, 4096 * 16));
  CK(hipMemset(ring, 0, alloc));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int grid = 2048;
  auto timeit = [&](auto launch) {
    for (int w = 0; w < 3; ++w) launch(w);
    CK(hipDeviceSynchronize());
    const int reps = 8;
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r) launch(r);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms * 1e3 / reps;
  };
  // footprint test: each launch moves 1 GiB, a ring of rb bytes, launches rotate over
  // (alloc / rb) disjoint regions, so nothing is re-used from one launch to the next
  // unless the region count is 1
  for (long rb : {1L << 30, 512L << 20, 256L << 20, 128L << 20}) {
    const long ri = rb / (ITEM * 16);
    for (long regions : {1L, alloc / rb}) {
      const double tw = timeit([&](int r) {
        hipLaunchKernelGGL(k_write, dim3(grid), dim3(256), 0, 0, ring + (r % regions) * ri * ITEM, ri, items);
      });
      const double tr = timeit([&](int r) {
        hipLaunchKernelGGL(k_read, dim3(grid), dim3(256), 0, 0, ring + (r % regions) * ri * ITEM, ri, items, sink);
      });
      std::printf("ring %5ld MiB x %2ld regions: write 1 GiB %7.1f us (%5.2f TB/s)  read 1 GiB %7.1f us (%5.2f TB/s)\n",
                  rb >> 20, regions, tw, total / (tw * 1e-6) / 1e12, tr, total / (tr * 1e-6) / 1e12);
    }
  }
  // one fresh pass (each launch a region untouched for >= 3 GiB of traffic)
  // of S bytes: does the launch's own footprint set the rate?
  for (long S : {128L << 20, 256L << 20, 512L << 20, 1L << 30}) {
    const long it = S / (ITEM * 16);
    const long regions = alloc / S;
    const double tw = timeit([&](int r) {
      hipLaunchKernelGGL(k_write, dim3(grid), dim3(256), 0, 0, ring + (r % regions) * it * ITEM, it, it);
    });
    const double tr = timeit([&](int r) {
      hipLaunchKernelGGL(k_read, dim3(grid), dim3(256), 0, 0, ring + (r % regions) * it * ITEM, it, it, sink);
    });
    std::printf("fresh single pass %5ld MiB: write %7.1f us (%5.2f TB/s)  read %7.1f us (%5.2f TB/s)\n", S >> 20, tw,
                S / (tw * 1e-6) / 1e12, tr, S / (tr * 1e-6) / 1e12);
  }
  // translation test: a single fresh pass over 1 GiB (regions rotate over 4 GiB),
  // optionally preceded (same stream, not timed separately) by a sparse touch of
  // that region: one load per 64 KiB or per 2 MiB
  {
    const long ri = items;
    for (long stride : {0L, 2L << 20, 64L << 10, 4L << 10}) {
      const double tw = timeit([&](int r) {
        double2* base = ring + (r % 4) * ri * ITEM;
        if (stride) hipLaunchKernelGGL(k_touch, dim3(256), dim3(256), 0, 0, base, total, stride, sink);
        hipLaunchKernelGGL(k_write, dim3(grid), dim3(256), 0, 0, base, ri, items);
      });
      const double tt = stride ? timeit([&](int r) {
        double2* base = ring + (r % 4) * ri * ITEM;
        hipLaunchKernelGGL(k_touch, dim3(256), dim3(256), 0, 0, base, total, stride, sink);
      }) : 0.0;
      const double tr = timeit([&](int r) {
        double2* base = ring + (r % 4) * ri * ITEM;
        if (stride) hipLaunchKernelGGL(k_touch, dim3(256), dim3(256), 0, 0, base, total, stride, sink);
        hipLaunchKernelGGL(k_read, dim3(grid), dim3(256), 0, 0, base, ri, items, sink);
      });
      std::printf("fresh 1 GiB, touch stride %8ld B (touch alone %6.1f us): write+touch %7.1f us, read+touch %7.1f us\n",
                  stride, tt, tw, tr);
    }
  }
  // a 4 GiB sweep in one launch
  {
    const long it4 = alloc / (ITEM * 16);
    const double tw = timeit([&](int) { hipLaunchKernelGGL(k_write, dim3(grid), dim3(256), 0, 0, ring, it4, it4); });
    const double tr = timeit([&](int) { hipLaunchKernelGGL(k_read, dim3(grid), dim3(256), 0, 0, ring, it4, it4, sink); });
    std::printf("4 GiB sweep: write %7.1f us (%5.2f TB/s)  read %7.1f us (%5.2f TB/s)\n", tw, alloc / (tw * 1e-6) / 1e12,
                tr, alloc / (tr * 1e-6) / 1e12);
  }
  for (long rb : {1L << 30, 256L << 20, 128L << 20, 64L << 20}) {
    const long ri = rb / (ITEM * 16);
    for (long lag : {512L, 2048L}) {
      if (lag >= ri) continue;
      const double t = timeit([&](int) { hipLaunchKernelGGL(k_rw, dim3(grid), dim3(256), 0, 0, ring, ri, items, lag, sink); });
      std::printf("rw ring %5ld MiB lag %5ld items (%4ld MiB): 1 GiB written + read %7.1f us (%5.2f TB/s moved)\n",
                  rb >> 20, lag, lag * ITEM * 16 >> 20, t, 2.0 * total / (t * 1e-6) / 1e12);
    }
  }
  return 0;
}
