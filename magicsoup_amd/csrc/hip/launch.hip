// Graph batching of the device core's launches (see launch.h).
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>

#include <cstdlib>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#include "hip_common.h"
#include "launch.h"

namespace py = pybind11;

namespace msd {
namespace {

constexpr int kMaxNodes = 96;       // a longer run is flushed in pieces
constexpr size_t kMaxGraphs = 512;  // distinct kernel sequences kept instantiated

struct Node {
  const void* f;
  dim3 g, b;
  unsigned lds;
  int a0, na;  // its arguments: entries [a0, a0 + na) of Batch::args
};

struct Arg {
  size_t off, size;
};

struct Batch {
  int depth = 0;
  hipStream_t st = nullptr;
  std::vector<Node> nodes;
  std::vector<Arg> args;
  std::vector<unsigned char> bytes;
};

struct Graph {
  hipGraph_t graph = nullptr;
  hipGraphExec_t exec = nullptr;
  std::vector<hipGraphNode_t> handles;
  std::vector<const void*> funcs;  // (collision check of the sequence hash)
  std::vector<dim3> blocks;
  // what each node holds now: grid, LDS bytes, argument bytes
  std::vector<dim3> grids;
  std::vector<unsigned> lds;
  std::vector<std::vector<unsigned char>> argv;
};

thread_local Batch t_batch;
std::mutex g_graphs_mu;  // (a call that released the GIL may flush next to another thread)
std::unordered_map<uint64_t, Graph> g_graphs;
int g_enabled = -1;  // -1: read MS_GRAPH_BATCH on first use (default off, see launch.h)
int g_min_nodes = 2;

struct Stats {
  long long graph_launches = 0, graph_nodes = 0, direct = 0, instantiated = 0, updated_nodes = 0, flushes = 0;
  long long sizes[kMaxNodes + 1] = {};  // flushes by batch length
} g_stats;

bool enabled() {
  if (g_enabled < 0) {
    const char* e = std::getenv("MS_GRAPH_BATCH");
    g_enabled = (e && e[0] == '1') ? 1 : 0;
  }
  return g_enabled == 1;
}

size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

void* arg_ptr(Batch& bt, int i) { return bt.bytes.data() + bt.args[i].off; }

void launch_direct(Batch& bt) {
  std::vector<void*> ptrs;
  for (const Node& n : bt.nodes) {
    ptrs.resize(n.na > 0 ? n.na : 1);
    for (int i = 0; i < n.na; ++i) ptrs[i] = arg_ptr(bt, n.a0 + i);
    MS_HIP_CHECK(hipLaunchKernel(n.f, n.g, n.b, ptrs.data(), n.lds, bt.st));
    ++g_stats.direct;
  }
}

uint64_t seq_hash(const Batch& bt, int dev) {
  uint64_t h = 1469598103934665603ull ^ (uint64_t)(unsigned)dev;
  auto mix = [&h](uint64_t v) {
    h ^= v + 0x9E3779B97F4A7C15ull + (h << 6) + (h >> 2);
    h *= 1099511628211ull;
  };
  mix(bt.nodes.size());
  for (const Node& n : bt.nodes) {
    mix(reinterpret_cast<uintptr_t>(n.f));
    mix(((uint64_t)n.b.x << 32) ^ ((uint64_t)n.b.y << 16) ^ n.b.z);
  }
  return h;
}

bool same_seq(const Graph& gr, const Batch& bt) {
  if (gr.funcs.size() != bt.nodes.size()) return false;
  for (size_t i = 0; i < bt.nodes.size(); ++i) {
    const dim3& b = gr.blocks[i];
    const Node& n = bt.nodes[i];
    if (gr.funcs[i] != n.f || b.x != n.b.x || b.y != n.b.y || b.z != n.b.z) return false;
  }
  return true;
}

void drop_graphs() {
  // (instantiated graphs may still be running: wait before destroying them; rare)
  MS_HIP_CHECK(hipDeviceSynchronize());
  for (auto& kv : g_graphs) {
    if (kv.second.exec) (void)hipGraphExecDestroy(kv.second.exec);
    if (kv.second.graph) (void)hipGraphDestroy(kv.second.graph);
  }
  g_graphs.clear();
}

hipKernelNodeParams params_of(Batch& bt, const Node& n, std::vector<void*>& ptrs) {
  ptrs.resize(n.na > 0 ? n.na : 1);
  for (int i = 0; i < n.na; ++i) ptrs[i] = arg_ptr(bt, n.a0 + i);
  hipKernelNodeParams p{};
  p.func = const_cast<void*>(n.f);
  p.gridDim = n.g;
  p.blockDim = n.b;
  p.sharedMemBytes = n.lds;
  p.kernelParams = ptrs.data();
  p.extra = nullptr;
  return p;
}

std::vector<unsigned char> arg_bytes(Batch& bt, const Node& n) {
  std::vector<unsigned char> v;
  for (int i = 0; i < n.na; ++i) {
    const unsigned char* p = static_cast<const unsigned char*>(arg_ptr(bt, n.a0 + i));
    v.insert(v.end(), p, p + bt.args[n.a0 + i].size);
  }
  return v;
}

bool args_equal(Batch& bt, const Node& n, const std::vector<unsigned char>& held) {
  size_t o = 0;
  for (int i = 0; i < n.na; ++i) {
    const size_t sz = bt.args[n.a0 + i].size;
    if (o + sz > held.size() || std::memcmp(held.data() + o, arg_ptr(bt, n.a0 + i), sz) != 0) return false;
    o += sz;
  }
  return o == held.size();
}

void launch_graph(Batch& bt) {
  int dev = 0;
  MS_HIP_CHECK(hipGetDevice(&dev));
  const uint64_t key = seq_hash(bt, dev);
  std::lock_guard<std::mutex> lk(g_graphs_mu);
  auto it = g_graphs.find(key);
  std::vector<void*> ptrs;
  if (it != g_graphs.end() && !same_seq(it->second, bt)) {
    // (a hash collision: launch directly rather than evict)
    launch_direct(bt);
    return;
  }
  if (it == g_graphs.end()) {
    if (g_graphs.size() >= kMaxGraphs) drop_graphs();
    Graph gr;
    MS_HIP_CHECK(hipGraphCreate(&gr.graph, 0));
    hipGraphNode_t prev = nullptr;
    for (const Node& n : bt.nodes) {
      hipKernelNodeParams p = params_of(bt, n, ptrs);
      hipGraphNode_t h = nullptr;
      MS_HIP_CHECK(hipGraphAddKernelNode(&h, gr.graph, prev ? &prev : nullptr, prev ? 1 : 0, &p));
      prev = h;
      gr.handles.push_back(h);
      gr.funcs.push_back(n.f);
      gr.blocks.push_back(n.b);
      gr.grids.push_back(n.g);
      gr.lds.push_back(n.lds);
      gr.argv.push_back(arg_bytes(bt, n));
    }
    MS_HIP_CHECK(hipGraphInstantiate(&gr.exec, gr.graph, nullptr, nullptr, 0));
    ++g_stats.instantiated;
    it = g_graphs.emplace(key, std::move(gr)).first;
  } else {
    Graph& gr = it->second;
    for (size_t i = 0; i < bt.nodes.size(); ++i) {
      const Node& n = bt.nodes[i];
      const dim3& g0 = gr.grids[i];
      if (g0.x == n.g.x && g0.y == n.g.y && g0.z == n.g.z && gr.lds[i] == n.lds && args_equal(bt, n, gr.argv[i]))
        continue;
      hipKernelNodeParams p = params_of(bt, n, ptrs);
      MS_HIP_CHECK(hipGraphExecKernelNodeSetParams(gr.exec, gr.handles[i], &p));
      gr.grids[i] = n.g;
      gr.lds[i] = n.lds;
      gr.argv[i] = arg_bytes(bt, n);
      ++g_stats.updated_nodes;
    }
  }
  MS_HIP_CHECK(hipGraphLaunch(it->second.exec, bt.st));
  ++g_stats.graph_launches;
  g_stats.graph_nodes += (long long)bt.nodes.size();
}

void clear(Batch& bt) {
  bt.nodes.clear();
  bt.args.clear();
  bt.bytes.clear();
}

}  // namespace

bool batch_recording() { return t_batch.depth > 0 && enabled(); }

void batch_enter() { ++t_batch.depth; }

void batch_flush() {
  Batch& bt = t_batch;
  if (bt.nodes.empty()) return;
  ++g_stats.flushes;
  ++g_stats.sizes[bt.nodes.size() <= (size_t)kMaxNodes ? bt.nodes.size() : kMaxNodes];
  try {
    if ((int)bt.nodes.size() < g_min_nodes) launch_direct(bt);
    else launch_graph(bt);
  } catch (...) {
    clear(bt);
    throw;
  }
  clear(bt);
}

void batch_exit(bool flush_now) {
  Batch& bt = t_batch;
  if (bt.depth == 1) {
    if (flush_now) {
      bt.depth = 0;
      batch_flush();
      return;
    }
    try {
      batch_flush();  // (leaving by an exception: what was recorded before it still goes out)
    } catch (...) {
    }
  }
  if (bt.depth > 0) --bt.depth;
}

void batch_record(const void* f, dim3 g, dim3 b, unsigned lds, hipStream_t st, void** args, const size_t* sizes,
                  const size_t* aligns, int nargs) {
  Batch& bt = t_batch;
  if (!bt.nodes.empty() && st != bt.st) batch_flush();  // (another stream: what came before goes first)
  bt.st = st;
  Node n{f, g, b, lds, (int)bt.args.size(), nargs};
  for (int i = 0; i < nargs; ++i) {
    const size_t off = align_up(bt.bytes.size(), aligns[i] < 16 ? aligns[i] : 16);
    bt.bytes.resize(off + sizes[i]);
    std::memcpy(bt.bytes.data() + off, args[i], sizes[i]);
    bt.args.push_back(Arg{off, sizes[i]});
  }
  bt.nodes.push_back(n);
  if ((int)bt.nodes.size() >= kMaxNodes) batch_flush();
}

void bind_launch(py::module_& m) {
  m.def("set_graph_batch", [](bool on, int min_nodes) {
    batch_flush();
    g_enabled = on ? 1 : 0;
    g_min_nodes = min_nodes < 1 ? 1 : min_nodes;
  }, py::arg("on"), py::arg("min_nodes") = 2,
        "batch the kernels of each native call into one hipGraph launch (min_nodes: shorter runs launch directly)");
  m.def("graph_batch", []() { return enabled(); });
  m.def("graph_batch_stats", []() {
    py::dict d;
    d["graph_launches"] = g_stats.graph_launches;
    d["graph_nodes"] = g_stats.graph_nodes;
    d["direct"] = g_stats.direct;
    d["instantiated"] = g_stats.instantiated;
    d["updated_nodes"] = g_stats.updated_nodes;
    d["flushes"] = g_stats.flushes;
    d["graphs"] = (long long)g_graphs.size();
    py::dict h;
    for (int i = 1; i <= kMaxNodes; ++i)
      if (g_stats.sizes[i]) h[py::int_(i)] = g_stats.sizes[i];
    d["batch_sizes"] = h;
    return d;
  }, "counters of the graph batching (launches, nodes, direct launches, instantiations, node updates)");
  m.def("graph_batch_reset", []() {
    batch_flush();
    std::lock_guard<std::mutex> lk(g_graphs_mu);
    g_stats = Stats{};
    drop_graphs();
  }, "drop every instantiated graph and zero the counters");
}

}  // namespace msd
