// Multi-GPU stereo mixdown over RCCL (SURVEY 8(b) ad_mixdown_reduce, 8(e)).
//
// The hot path shards by channel group: one process per GPU convolves its
// own channels with no data-path collective, and the only exchange is one
// sum-reduce of the per-rank stereo partial mixes to the root rank over
// xGMI.  The communicator is a plain RCCL communicator created from a unique
// id (the caller moves the 128 id bytes between its processes), so a Go host
// can shard through cgo without torch.distributed.
//
// librccl.so.1 is dlopen'ed on first use: a single-GPU caller never needs it,
// and in a process that already holds RCCL (PyTorch's bundled copy has the
// same soname) the loader hands back that copy, so only one RCCL runs.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <mutex>
#include <string>

#include "ad_common.hpp"
#include "conv_kernels.hpp"

using namespace adsp;

namespace {

struct Rccl {
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRank) comm_init_rank = nullptr;
  decltype(&ncclCommDestroy) comm_destroy = nullptr;
  decltype(&ncclReduce) reduce = nullptr;
  decltype(&ncclGroupStart) group_start = nullptr;
  decltype(&ncclGroupEnd) group_end = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
  std::string load_error;
};

const Rccl& rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) {
      const char* e = dlerror();
      r.load_error = std::string("cannot load librccl.so.1: ") + (e ? e : "?");
      return;
    }
    auto sym = [&](const char* name) {
      void* p = dlsym(h, name);
      if (!p && r.load_error.empty()) r.load_error = std::string("librccl.so.1 lacks ") + name;
      return p;
    };
    r.get_unique_id = reinterpret_cast<decltype(r.get_unique_id)>(sym("ncclGetUniqueId"));
    r.comm_init_rank = reinterpret_cast<decltype(r.comm_init_rank)>(sym("ncclCommInitRank"));
    r.comm_destroy = reinterpret_cast<decltype(r.comm_destroy)>(sym("ncclCommDestroy"));
    r.reduce = reinterpret_cast<decltype(r.reduce)>(sym("ncclReduce"));
    r.group_start = reinterpret_cast<decltype(r.group_start)>(sym("ncclGroupStart"));
    r.group_end = reinterpret_cast<decltype(r.group_end)>(sym("ncclGroupEnd"));
    r.error_string = reinterpret_cast<decltype(r.error_string)>(sym("ncclGetErrorString"));
  });
  if (!r.load_error.empty()) AD_FAIL(AD_ERR_DEVICE, r.load_error);
  return r;
}

#define AD_NCCL(expr)                                                                             \
  do {                                                                                            \
    const ncclResult_t _r = (expr);                                                               \
    if (_r != ncclSuccess)                                                                        \
      AD_FAIL(AD_ERR_DEVICE, std::string(#expr) + ": " + rccl().error_string(_r));                \
  } while (0)

}  // namespace

struct ad_comm {
  ncclComm_t comm = nullptr;
  int rank = 0, size = 1, device = 0;
};

extern "C" {

int ad_comm_get_unique_id(uint8_t id[AD_COMM_ID_BYTES]) {
  return guard([&] {
    if (!id) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "null id buffer");
    static_assert(sizeof(ncclUniqueId) == AD_COMM_ID_BYTES, "RCCL unique id size");
    ncclUniqueId u;
    AD_NCCL(rccl().get_unique_id(&u));
    std::memcpy(id, &u, sizeof(u));
  });
}

int ad_comm_create(const uint8_t id[AD_COMM_ID_BYTES], int nranks, int rank, int device, ad_comm** out) {
  if (out) *out = nullptr;
  return guard([&] {
    if (!id || !out) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "null argument");
    if (nranks < 1 || rank < 0 || rank >= nranks) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "bad rank / world size");
    const int dev = pick_device(device);
    DeviceScope ds(dev);
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof(u));
    auto* c = new ad_comm();
    c->rank = rank;
    c->size = nranks;
    c->device = dev;
    const ncclResult_t r = rccl().comm_init_rank(&c->comm, nranks, u, rank);
    if (r != ncclSuccess) {
      delete c;
      AD_FAIL(AD_ERR_DEVICE, std::string("ncclCommInitRank: ") + rccl().error_string(r));
    }
    *out = c;
  });
}

void ad_comm_destroy(ad_comm* c) {
  if (!c) return;
  if (c->comm) {
    try {
      (void)rccl().comm_destroy(c->comm);
    } catch (...) {
    }
  }
  delete c;
}

int ad_comm_rank(const ad_comm* c) { return c ? c->rank : -1; }
int ad_comm_size(const ad_comm* c) { return c ? c->size : 0; }

int ad_mixdown_reduce(ad_comm* c, const double* d_chan, int channels, int64_t stride, int64_t len, int first_parity,
                      double* d_mix, int64_t mix_stride, int root, void* stream) {
  return guard([&] {
    if (!c || !c->comm) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "null communicator");
    if (len <= 0) AD_FAIL(AD_ERR_EMPTY_INPUT, "empty mixdown");
    if (!d_mix) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "mixdown: null mix buffer");
    if (mix_stride < len) AD_FAIL(AD_ERR_LENGTH_MISMATCH, "mixdown: mix stride shorter than the length");
    if (root < 0 || root >= c->size) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "mixdown: root out of range");
    if (channels < 0) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "mixdown: negative channel count");
    DeviceScope ds(c->device);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (channels > 0) {
      if (!d_chan) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "mixdown: null channel buffer");
      if (channels > 1 && stride < len) AD_FAIL(AD_ERR_LENGTH_MISMATCH, "mixdown: channel stride shorter than len");
      launch_mixdown(d_chan, channels, stride, len, d_mix, mix_stride, first_parity, s);
      AD_HIP(hipGetLastError());
    }
    const Rccl& r = rccl();
    if (mix_stride == len) {  // L and R rows are contiguous: one reduce
      AD_NCCL(r.reduce(d_mix, d_mix, (size_t)(2 * len), ncclFloat64, ncclSum, root, c->comm, s));
    } else {
      AD_NCCL(r.group_start());
      AD_NCCL(r.reduce(d_mix, d_mix, (size_t)len, ncclFloat64, ncclSum, root, c->comm, s));
      AD_NCCL(r.reduce(d_mix + mix_stride, d_mix + mix_stride, (size_t)len, ncclFloat64, ncclSum, root, c->comm, s));
      AD_NCCL(r.group_end());
    }
  });
}

}  // extern "C"
