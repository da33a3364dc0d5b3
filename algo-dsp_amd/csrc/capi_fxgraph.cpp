// Batched effect-chain graph runtime: `channels` copies of one effectchain
// graph (dsp/effectchain) run together on the GPU, one lane per channel.
//
// Reference semantics (chain_process.go:11-319): nodes run in topological
// order; a node's input is the average of its parents' outputs
// (mixParentEdgesInto, :295-318: zeros without parents, a copy for one, the
// sum in edge order times 1/k for k), split-freq nodes write an LR4 low and
// high band (crossover.ProcessBlock, filter/crossover/crossover.go:80-94) that
// their consumers read by port, _output and bypassed nodes only mix, and every
// other node processes its buffer in place.  The output node's buffer is the
// result.
//
// Compilation (ad_fx_graph_create) turns the node list into device ops:
//   * a node whose single parent port feeds nobody else takes over that
//     buffer (no copy; in-place processing as the reference's copy-then-
//     process gives the same values);
//   * consecutive in-place nodes on one buffer fuse into one effect-chain
//     launch when their stages come in the kernel's order: biquad sections
//     (consecutive filter nodes concatenate: per sample, chain after chain),
//     then one compressor/limiter, then one Freeverb.  Per-sample fusion is
//     exact (every stage is causal and sees only its predecessor's output of
//     the same sample), so results are bit-identical with node-by-node runs;
//   * fan-in mixes are one kernel (k_fx_mix) in the reference's summation
//     order; the split-freq low band runs in place on the node's buffer and
//     the high band on a copy;
//   * independent branches run concurrently on up to 8 streams (schedule()).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <memory>
#include <vector>

#include "ad_common.hpp"
#include "dsp_kernels.hpp"

using namespace adsp;

namespace adsp {
void fx_chain_allow_staged(ad_fx_chain* h, bool on);  // capi_dsp.cpp
}

namespace {

void ck(int rc) {
  if (rc != AD_OK) AD_FAIL(rc, ad_last_error());
}

struct ChainDel {
  void operator()(ad_fx_chain* c) const { ad_fx_chain_destroy(c); }
};
using ChainPtr = std::unique_ptr<ad_fx_chain, ChainDel>;

struct ConvDel {
  void operator()(ad_conv* c) const { ad_conv_destroy(c); }
};
using ConvPtr = std::unique_ptr<ad_conv, ConvDel>;

struct FxOp {
  enum Kind { ZERO, COPY, MIX, CHAIN, CONV } kind;
  int dst = -1;                 // buffer id (written; CHAIN / CONV: read and written in place)
  std::vector<int> srcs;        // COPY / MIX: buffers read
  ad_fx_chain* chain = nullptr;   // CHAIN
  ad_conv* conv = nullptr;        // CONV (many-channel convolution reverb)
  // schedule (see schedule()): lane 0 is the caller's stream
  int lane = 0;
  std::vector<int> waits;  // ops on other lanes this op waits for
  bool signal = false;     // another lane waits for this op
};

// Stage group under construction for the fusion pass.
struct Group {
  std::vector<double> sections;  // [nsec][6]
  const ad_fx_node* dyn = nullptr;  // the dynamics node (compressor / limiter / expander / gate)
  const double* verb = nullptr;
  bool open = false;
  int buf = -1;
  int level() const { return verb ? 3 : (dyn ? 2 : (sections.empty() ? 0 : 1)); }
};

}  // namespace

struct ad_fx_graph {
  int device = 0, channels = 0;
  hipStream_t stream = nullptr;
  int nbuf = 1;          // buffer 0 = the caller's block
  int out_buf = 0;
  std::vector<FxOp> ops;
  std::vector<ChainPtr> chains;
  std::vector<ConvPtr> convs;
  DevBuf<double> pool;   // buffers 1..nbuf-1, [nbuf-1][channels][cap]
  int64_t cap = 0;
  DevBuf<double> work;   // host-call staging
  int lanes_used = 1;
  std::vector<int> lane_tail;        // last op of lanes 1..
  hipStream_t lane[8] = {};          // lanes 1..: internal streams
  hipEvent_t start_ev = nullptr;
  std::vector<hipEvent_t> op_ev;     // per op (signalling ops only)
  ~ad_fx_graph() {
    for (auto& e : op_ev)
      if (e) (void)hipEventDestroy(e);
    if (start_ev) (void)hipEventDestroy(start_ev);
    for (auto& l : lane)
      if (l) {
        (void)hipStreamSynchronize(l);
        (void)lib_stream_destroy(l);
      }
    chains.clear();
    convs.clear();
    if (stream) {
      (void)hipStreamSynchronize(stream);
      (void)lib_stream_destroy(stream);
    }
  }
};

namespace {

ad_fx_chain* new_chain(ad_fx_graph* g) {
  ad_fx_chain* c = nullptr;
  ck(ad_fx_chain_create(g->channels, g->device, &c));
  g->chains.emplace_back(c);
  return c;
}

void flush(ad_fx_graph* g, Group& gr) {
  if (!gr.open) return;
  if (gr.level() > 0) {
    ad_fx_chain* c = new_chain(g);
    if (!gr.sections.empty()) ck(ad_fx_chain_set_eq(c, gr.sections.data(), (int)(gr.sections.size() / kSecStride), 0));
    if (gr.dyn) {
      if (gr.dyn->dyn_mode == 0)
        ck(ad_fx_chain_set_compressor(c, gr.dyn->comp));
      else
        ck(ad_fx_chain_set_expander(c, gr.dyn->comp, gr.dyn->dyn_mode == 2, gr.dyn->dyn_range_db,
                                    gr.dyn->dyn_hold_ms));
    }
    if (gr.verb) ck(ad_fx_chain_set_freeverb(c, gr.verb[0], gr.verb[1], gr.verb[2], gr.verb[3], gr.verb[4]));
    FxOp op{FxOp::CHAIN};
    op.dst = gr.buf;
    op.chain = c;
    g->ops.push_back(op);
  }
  gr = Group{};
}

void compile(ad_fx_graph* g, const ad_fx_node* nodes, int n) {
  if (n < 2 || nodes[0].type != AD_FXN_INPUT) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "fx graph: node 0 must be the input");
  // consumers of each (node, port)
  std::vector<int> uses((size_t)n * 2, 0);
  int out_node = -1;
  for (int i = 0; i < n; ++i) {
    const ad_fx_node& d = nodes[i];
    if (d.type < AD_FXN_INPUT || d.type > AD_FXN_CONV_REVERB)
      AD_FAIL(AD_ERR_UNKNOWN_EFFECT, "fx graph: node type not supported by the GPU runtime");
    if (d.type == AD_FXN_INPUT && i != 0) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "fx graph: more than one input node");
    if (d.type == AD_FXN_OUTPUT) {
      if (out_node >= 0) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "fx graph: more than one output node");
      out_node = i;
    }
    if (d.n_parents < 0 || d.n_parents > AD_FX_MAX_PARENTS || (d.n_parents > 0 && !d.parents))
      AD_FAIL(AD_ERR_INVALID_ARGUMENT, "fx graph: bad parent list");
    for (int k = 0; k < d.n_parents; ++k) {
      const int p = d.parents[k];
      const int port = d.parent_ports ? d.parent_ports[k] : 0;
      if (p < 0 || p >= i) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "fx graph: parents must precede their node (topological order)");
      if (port != 0 && !(port == 1 && nodes[p].type == AD_FXN_SPLIT_FREQ))
        AD_FAIL(AD_ERR_INVALID_ARGUMENT, "fx graph: port 1 exists only on split-freq nodes");
      uses[(size_t)p * 2 + port]++;
    }
    if (d.type == AD_FXN_BIQUAD && (d.nsec < 0 || (d.nsec > 0 && !d.sections)))
      AD_FAIL(AD_ERR_INVALID_ARGUMENT, "fx graph: filter node without sections");
    if (d.type == AD_FXN_SPLIT_FREQ && (d.nsec <= 0 || !d.sections || d.nsec2 <= 0 || !d.sections2))
      AD_FAIL(AD_ERR_INVALID_ARGUMENT, "fx graph: split-freq node needs LP and HP sections");
    if (d.type == AD_FXN_COMPRESSOR && !d.comp) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "fx graph: compressor without config");
    if (d.type == AD_FXN_CONV_REVERB && !d.bypassed && (!d.ir || d.ir_len <= 0))
      AD_FAIL(AD_ERR_EMPTY_IMPULSE_RESPONSE, "fx graph: reverb-conv node without an impulse response");
    if (d.type == AD_FXN_COMPRESSOR && (d.dyn_mode < 0 || d.dyn_mode > 2))
      AD_FAIL(AD_ERR_INVALID_ARGUMENT, "fx graph: bad dynamics mode");
  }
  if (out_node < 0) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "fx graph: no output node");

  std::vector<int> buf_of((size_t)n * 2, -1);  // buffer id of (node, port)
  buf_of[0] = 0;
  Group gr;
  for (int i = 1; i < n; ++i) {
    const ad_fx_node& d = nodes[i];
    // ---- the node's input (mixParentEdgesInto)
    int b;
    const int port0 = d.n_parents ? (d.parent_ports ? d.parent_ports[0] : 0) : 0;
    if (d.n_parents == 1 && uses[(size_t)d.parents[0] * 2 + port0] == 1) {
      b = buf_of[(size_t)d.parents[0] * 2 + port0];  // sole consumer: take the buffer over
    } else {
      b = g->nbuf++;
      FxOp op{d.n_parents == 0 ? FxOp::ZERO : (d.n_parents == 1 ? FxOp::COPY : FxOp::MIX)};
      op.dst = b;
      for (int k = 0; k < d.n_parents; ++k)
        op.srcs.push_back(buf_of[(size_t)d.parents[k] * 2 + (d.parent_ports ? d.parent_ports[k] : 0)]);
      flush(g, gr);
      g->ops.push_back(op);
    }
    if (gr.open && gr.buf != b) flush(g, gr);
    buf_of[(size_t)i * 2] = b;

    // ---- the node itself
    if (d.type == AD_FXN_SPLIT_FREQ) {
      flush(g, gr);
      // high band = HP chain on a copy, low band = LP chain in place
      const int hb = g->nbuf++;
      FxOp cp{FxOp::COPY};
      cp.dst = hb;
      cp.srcs.push_back(b);
      g->ops.push_back(cp);
      FxOp lo{FxOp::CHAIN};
      lo.dst = b;
      lo.chain = new_chain(g);
      ck(ad_fx_chain_set_eq(lo.chain, d.sections, d.nsec, 0));
      g->ops.push_back(lo);
      FxOp hi{FxOp::CHAIN};
      hi.dst = hb;
      hi.chain = new_chain(g);
      ck(ad_fx_chain_set_eq(hi.chain, d.sections2, d.nsec2, 0));
      g->ops.push_back(hi);
      buf_of[(size_t)i * 2 + 1] = hb;
      continue;
    }
    if (d.type == AD_FXN_OUTPUT || d.type == AD_FXN_PASS || d.bypassed) continue;
    if (d.type == AD_FXN_CONV_REVERB) {
      flush(g, gr);
      ad_conv* cr = nullptr;
      ck(ad_conv_reverb_multi_create(d.ir, d.ir_len, d.conv_min_order, g->channels, g->device, &cr));
      g->convs.emplace_back(cr);
      ck(ad_conv_reverb_set_wet_dry(cr, d.conv_wet, d.conv_dry));
      FxOp op{FxOp::CONV};
      op.dst = b;
      op.conv = cr;
      g->ops.push_back(op);
      continue;
    }
    const int lvl = d.type == AD_FXN_BIQUAD ? 1 : (d.type == AD_FXN_COMPRESSOR ? 2 : 3);
    if (gr.open && (lvl < gr.level() || (lvl == gr.level() && lvl > 1))) flush(g, gr);
    gr.open = true;
    gr.buf = b;
    if (lvl == 1) {
      gr.sections.insert(gr.sections.end(), d.sections, d.sections + (size_t)d.nsec * kSecStride);
    } else if (lvl == 2) {
      gr.dyn = &d;
    } else {
      gr.verb = d.verb;
    }
  }
  flush(g, gr);
  g->out_buf = buf_of[(size_t)out_node * 2];
  if (g->out_buf != 0) {  // copyOutputToBlock (chain_process.go:274-283)
    FxOp op{FxOp::COPY};
    op.dst = 0;
    op.srcs.push_back(g->out_buf);
    g->ops.push_back(op);
  }
}

// Independent branches run concurrently: every chain op is only
// ceil(channels/64) workgroups (one lane per channel, serial in time), so the
// GPU has room for all of them at once.  Dependencies come from the buffers
// each op reads and writes (read-after-write, write-after-read and
// write-after-write); an op continues the lane of a dependency that is the
// lane's last op, otherwise it opens a new lane (at most kLanes), and it
// waits on events of dependencies on other lanes.
constexpr int kLanes = 8;
void schedule(ad_fx_graph* g) {
  const int nb = g->nbuf;
  std::vector<int> last_writer(nb, -1);
  std::vector<std::vector<int>> readers(nb);
  std::vector<int> tail(kLanes, -1);  // last op of each lane
  int used = 1;
  for (int i = 0; i < (int)g->ops.size(); ++i) {
    FxOp& op = g->ops[i];
    std::vector<int> reads = op.srcs;
    if (op.kind == FxOp::CHAIN || op.kind == FxOp::CONV) reads.push_back(op.dst);
    std::vector<int> deps;
    for (int b : reads)
      if (last_writer[b] >= 0) deps.push_back(last_writer[b]);
    if (last_writer[op.dst] >= 0) deps.push_back(last_writer[op.dst]);
    for (int r : readers[op.dst]) deps.push_back(r);
    std::sort(deps.begin(), deps.end());
    deps.erase(std::unique(deps.begin(), deps.end()), deps.end());
    deps.erase(std::remove(deps.begin(), deps.end(), i), deps.end());
    int lane = -1;
    for (int d : deps)
      if (tail[g->ops[d].lane] == d) {
        lane = g->ops[d].lane;
        break;
      }
    if (lane < 0) {
      if (deps.empty() && tail[0] < 0) lane = 0;
      else if (used < kLanes) lane = used++;
      else lane = i % kLanes;
    }
    op.lane = lane;
    for (int d : deps)
      if (g->ops[d].lane != lane) {
        op.waits.push_back(d);
        g->ops[d].signal = true;
      }
    tail[lane] = i;
    for (int b : reads) readers[b].push_back(i);
    readers[op.dst].clear();
    last_writer[op.dst] = i;
  }
  // the caller's stream (lane 0) waits for every other lane's last op
  g->lanes_used = used;
  for (FxOp& op : g->ops)
    if (op.kind == FxOp::CHAIN) adsp::fx_chain_allow_staged(op.chain, used == 1);
  for (int l = 1; l < used; ++l)
    if (tail[l] >= 0) {
      g->ops[tail[l]].signal = true;
      g->lane_tail.push_back(tail[l]);
    }
}

double* buf_ptr(ad_fx_graph* g, int b, double* d0) {
  return b == 0 ? d0 : g->pool.p + (size_t)(b - 1) * g->channels * g->cap;
}

void run(ad_fx_graph* g, double* d0, int64_t stride0, int64_t n, hipStream_t s) {
  if (n == 0) return;
  if (g->nbuf > 1 && n > g->cap) {
    AD_HIP(hipStreamSynchronize(s));
    for (int l = 1; l < g->lanes_used; ++l) AD_HIP(hipStreamSynchronize(g->lane[l]));
    g->cap = n;
    g->pool.alloc((size_t)(g->nbuf - 1) * g->channels * g->cap);
  }
  auto st = [&](int b) { return b == 0 ? stride0 : g->cap; };
  auto lane_stream = [&](int l) { return l == 0 ? s : g->lane[l]; };
  if (g->lanes_used > 1) {  // the other lanes start after the caller's prior work
    AD_HIP(hipEventRecord(g->start_ev, s));
    for (int l = 1; l < g->lanes_used; ++l) AD_HIP(hipStreamWaitEvent(g->lane[l], g->start_ev, 0));
  }
  for (size_t i = 0; i < g->ops.size(); ++i) {
    const FxOp& op = g->ops[i];
    hipStream_t ls = lane_stream(op.lane);
    for (int w : op.waits) AD_HIP(hipStreamWaitEvent(ls, g->op_ev[w], 0));
    double* dst = buf_ptr(g, op.dst, d0);
    switch (op.kind) {
      case FxOp::ZERO:
        AD_HIP(hipMemset2DAsync(dst, st(op.dst) * 8, 0, n * 8, g->channels, ls));
        break;
      case FxOp::COPY:
        AD_HIP(hipMemcpy2DAsync(dst, st(op.dst) * 8, buf_ptr(g, op.srcs[0], d0), st(op.srcs[0]) * 8, n * 8,
                                g->channels, hipMemcpyDeviceToDevice, ls));
        break;
      case FxOp::MIX: {
        FxMixArgs m{};
        m.nsrc = (int)op.srcs.size();
        for (int k = 0; k < m.nsrc; ++k) {
          m.src[k] = buf_ptr(g, op.srcs[k], d0);
          m.src_stride[k] = st(op.srcs[k]);
        }
        m.dst = dst;
        m.dst_stride = st(op.dst);
        m.n = n;
        m.channels = g->channels;
        launch_fx_mix(m, ls);
        AD_HIP(hipGetLastError());
        break;
      }
      case FxOp::CHAIN:
        ck(ad_fx_chain_process_device(op.chain, dst, st(op.dst), n, ls));
        break;
      case FxOp::CONV:
        ck(ad_conv_reverb_multi_process_device(op.conv, dst, st(op.dst), n, ls));
        break;
    }
    if (op.signal) AD_HIP(hipEventRecord(g->op_ev[i], ls));
  }
  for (int t : g->lane_tail) AD_HIP(hipStreamWaitEvent(s, g->op_ev[t], 0));
}

template <class Fn>
int graph_guard(ad_fx_graph* g, Fn&& fn) {
  return guard([&] {
    if (!g) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "null fx graph handle");
    DeviceScope ds(g->device);
    fn();
  });
}

}  // namespace

extern "C" {

int ad_fx_graph_create(const ad_fx_node* nodes, int n_nodes, int channels, int device, ad_fx_graph** out) {
  if (out) *out = nullptr;
  ad_fx_graph* raw = nullptr;
  const int rc = guard([&] {
    if (!nodes || n_nodes <= 0) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "fx graph: no nodes");
    if (channels <= 0) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "channels must be positive");
    const int dev = pick_device(device);
    DeviceScope ds(dev);
    std::unique_ptr<ad_fx_graph> g(new ad_fx_graph());
    g->device = dev;
    g->channels = channels;
    AD_HIP(lib_stream_create(&g->stream));
    compile(g.get(), nodes, n_nodes);
    schedule(g.get());
    for (int l = 1; l < g->lanes_used; ++l) AD_HIP(lib_stream_create(&g->lane[l]));
    AD_HIP(hipEventCreateWithFlags(&g->start_ev, hipEventDisableTiming));
    g->op_ev.assign(g->ops.size(), nullptr);
    for (size_t i = 0; i < g->ops.size(); ++i)
      if (g->ops[i].signal) AD_HIP(hipEventCreateWithFlags(&g->op_ev[i], hipEventDisableTiming));
    raw = g.release();
  });
  if (rc == AD_OK && out) *out = raw;
  return rc;
}

int ad_fx_graph_op_count(const ad_fx_graph* g, int* launches, int* buffers, int* lanes) {
  if (!g) return AD_ERR_INVALID_ARGUMENT;
  if (launches) *launches = (int)g->ops.size();
  if (buffers) *buffers = g->nbuf;
  if (lanes) *lanes = g->lanes_used;
  return AD_OK;
}

int ad_fx_graph_process_device(ad_fx_graph* g, double* d_buf, int64_t stride, int64_t n, void* stream) {
  return graph_guard(g, [&] {
    if (n < 0 || stride < n) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "bad buffer geometry");
    run(g, d_buf, stride, n, reinterpret_cast<hipStream_t>(stream));
  });
}

int ad_fx_graph_process(ad_fx_graph* g, double* buf, int64_t n) {
  return graph_guard(g, [&] {
    if (n < 0 || (n > 0 && !buf)) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "bad buffer");
    if (n == 0) return;  // Chain.Process: an empty block is a no-op (chain_process.go:12-14)
    const size_t bytes = (size_t)g->channels * n * sizeof(double);
    g->work.reserve((size_t)g->channels * n);
    AD_HIP(hipMemcpyAsync(g->work.p, buf, bytes, hipMemcpyHostToDevice, g->stream));
    run(g, g->work.p, n, n, g->stream);
    AD_HIP(hipMemcpyAsync(buf, g->work.p, bytes, hipMemcpyDeviceToHost, g->stream));
    AD_HIP(hipStreamSynchronize(g->stream));
  });
}

int ad_fx_graph_reset(ad_fx_graph* g) {
  return graph_guard(g, [&] {
    for (auto& c : g->chains) ck(ad_fx_chain_reset(c.get()));
    for (auto& c : g->convs) ck(ad_conv_reset(c.get()));
  });
}

void ad_fx_graph_destroy(ad_fx_graph* g) {
  if (!g) return;
  const int dev = g->device;
  int cur = -1;
  (void)hipGetDevice(&cur);
  if (cur != dev) (void)hipSetDevice(dev);
  delete g;
  if (cur >= 0 && cur != dev) (void)hipSetDevice(cur);
}

}  // extern "C"
