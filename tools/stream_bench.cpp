// Per-block latency of the streaming host-buffer ABI without any Python in
// the loop (what a cgo caller sees, modulo cgo's ~100 ns call overhead).
//   stream_bench [K=16384] [B=4096] [blocks=4096] [kind=ols|pc] [minOrder=7] [pace_us=0]
// pace_us > 0: the caller sleeps between calls (a real-time caller's period),
// so the per-call latency includes whatever a paced call pays.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "algodsp.h"

int main(int argc, char** argv) {
  const long K = argc > 1 ? atol(argv[1]) : 16384;
  const long B = argc > 2 ? atol(argv[2]) : 4096;
  const long nb = argc > 3 ? atol(argv[3]) : 4096;
  const bool pc = argc > 4 && !strcmp(argv[4], "pc");
  const int min_order = argc > 5 ? atoi(argv[5]) : 7;
  const long pace_us = argc > 6 ? atol(argv[6]) : 0;
  std::vector<double> h(K), x(B), y(B);
  for (long i = 0; i < K; ++i) h[i] = std::exp(-1e-4 * i) * std::sin(0.37 * i);
  for (long i = 0; i < B; ++i) x[i] = std::sin(0.01 * i);
  ad_conv* c = nullptr;
  int rc = pc ? ad_conv_partitioned_create(h.data(), K, min_order, 13, 0, &c)
              : ad_conv_stream_ols_create(h.data(), K, B, 0, &c);
  if (rc) {
    fprintf(stderr, "create failed %d: %s\n", rc, ad_last_error());
    return 1;
  }
  auto call = [&] {
    return pc ? ad_conv_partitioned_process_block(c, x.data(), B, y.data(), B)
              : ad_conv_process_block(c, x.data(), B, y.data(), B);
  };
  for (int i = 0; i < 64; ++i) call();
  std::vector<double> lat(nb);
  const auto t0 = std::chrono::steady_clock::now();
  double busy = 0;
  for (long i = 0; i < nb; ++i) {
    if (pace_us > 0) std::this_thread::sleep_for(std::chrono::microseconds(pace_us));
    const auto a = std::chrono::steady_clock::now();
    if ((rc = call())) {
      fprintf(stderr, "process failed %d: %s\n", rc, ad_last_error());
      return 1;
    }
    lat[i] = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a).count();
    busy += lat[i];
  }
  const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  std::vector<double> s = lat;
  std::sort(s.begin(), s.end());
  printf("{\"kind\": \"%s\", \"K\": %ld, \"B\": %ld, \"blocks\": %ld, \"pace_us\": %ld, "
         "\"Msamples_per_s\": %.3f, \"us_per_block_mean\": %.2f, \"p50\": %.2f, \"p99\": %.2f}\n",
         pc ? "partitioned" : "streaming_ols", K, B, nb, pace_us, nb * B / (busy * 1e-6) / 1e6, busy / nb, s[nb / 2],
         s[(size_t)(nb * 0.99)]);
  ad_conv_destroy(c);
  return 0;
}
