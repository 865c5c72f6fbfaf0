// Host half of libsem_hip.so: node orderings of a cell-node map.
//
// DOFManager(mesh, ..., rcm_order=True) renumbers the mesh nodes by reverse
// Cuthill-McKee on the graph with an edge between every two nodes of a cell
// (sem/discrete.py:169-178: _get_connectivity_graph builds that boolean CSR
// graph, scipy.sparse.csgraph.reverse_cuthill_mckee(graph, True) orders it).
// That graph has sum_e nloc^2 entries -- 5.5e9 at 1024^2 cells, p = 8 -- and
// does not fit a host; these functions run the same algorithm on the cell map
// itself (node -> cells CSR, neighbours = union of the nodes of a node's
// cells, which is the graph's row), in O(nodes x cells-per-node x nloc):
//
//   degree(i) = |row i| + 1  (the row holds the diagonal, which scipy's
//               _node_degrees counts twice);
//   seeds     = argsort(degree), taken from the caller so that the tie order
//               is numpy's own (the reference's argsort, on the same host);
//   order     = breadth-first search from each unvisited seed in seed order;
//               the unvisited neighbours of each node are appended in
//               increasing node id (the CSR column order) and the appended
//               block is then stably sorted by degree (scipy's insertion
//               sort); RCM = order reversed (the caller reverses).
//
// tests/test_order.py checks the result equal to scipy's on the reference's
// own graph.
#include <algorithm>
#include <cstdint>
#include <string>
#include <thread>
#include <vector>

#include "sem_internal.h"

namespace {

struct NodeCells {
  std::vector<int64_t> ptr;
  std::vector<uint32_t> cells;
};

int node_cells(const uint32_t* cells, int64_t n_cells, int nloc, int64_t n_node, NodeCells& nc) {
  nc.ptr.assign((size_t)n_node + 1, 0);
  for (int64_t t = 0; t < n_cells * nloc; ++t) {
    if (cells[t] >= (uint64_t)n_node) return sem::fail(SEM_E_INVALID, "cell map references node >= n_node");
    nc.ptr[(size_t)cells[t] + 1]++;
  }
  for (int64_t i = 0; i < n_node; ++i) nc.ptr[(size_t)i + 1] += nc.ptr[(size_t)i];
  nc.cells.resize((size_t)nc.ptr[(size_t)n_node]);
  std::vector<int64_t> fill(nc.ptr.begin(), nc.ptr.end() - 1);
  for (int64_t e = 0; e < n_cells; ++e)
    for (int k = 0; k < nloc; ++k) {
      const uint32_t v = cells[e * nloc + k];
      const int64_t at = fill[v]++;
      // one entry per (node, cell) pair: a node listed twice in a cell counts once
      if (at > nc.ptr[v] && nc.cells[(size_t)at - 1] == (uint32_t)e) {
        --fill[v];
        continue;
      }
      nc.cells[(size_t)at] = (uint32_t)e;
    }
  // compact the dropped duplicates
  std::vector<int64_t> ptr2((size_t)n_node + 1, 0);
  int64_t w = 0;
  for (int64_t i = 0; i < n_node; ++i) {
    const int64_t b = nc.ptr[(size_t)i];
    for (int64_t t = b; t < fill[(size_t)i]; ++t) nc.cells[(size_t)w++] = nc.cells[(size_t)t];
    ptr2[(size_t)i + 1] = w;
  }
  nc.cells.resize((size_t)w);
  nc.ptr.swap(ptr2);
  return SEM_OK;
}

// row i of the cell-pair graph (sorted, unique) into buf
void graph_row(const NodeCells& nc, const uint32_t* cells, int nloc, int64_t i,
               std::vector<uint32_t>& buf) {
  buf.clear();
  for (int64_t t = nc.ptr[(size_t)i]; t < nc.ptr[(size_t)i + 1]; ++t) {
    const uint32_t* c = cells + (int64_t)nc.cells[(size_t)t] * nloc;
    buf.insert(buf.end(), c, c + nloc);
  }
  std::sort(buf.begin(), buf.end());
  buf.erase(std::unique(buf.begin(), buf.end()), buf.end());
}

int n_threads() {
  const unsigned h = std::thread::hardware_concurrency();
  return (int)std::max(1u, std::min(16u, h ? h : 1u));
}

}  // namespace

extern "C" {

int sem_node_degrees(const uint32_t* cells, int64_t n_cells, int nloc, int64_t n_node,
                     int32_t* degree) {
  if (!cells || !degree || n_cells < 0 || nloc < 1 || n_node < 1)
    return sem::fail(SEM_E_INVALID, "sem_node_degrees: invalid arguments");
  NodeCells nc;
  if (int rc = node_cells(cells, n_cells, nloc, n_node, nc)) return rc;
  const int nt = n_threads();
  std::vector<std::thread> th;
  for (int t = 0; t < nt; ++t)
    th.emplace_back([&, t] {
      std::vector<uint32_t> buf;
      for (int64_t i = t; i < n_node; i += nt) {
        graph_row(nc, cells, nloc, i, buf);
        // an isolated node has an empty row (no diagonal entry either)
        degree[i] = buf.empty() ? 0 : (int32_t)buf.size() + 1;
      }
    });
  for (auto& x : th) x.join();
  return SEM_OK;
}

int sem_cuthill_mckee(const uint32_t* cells, int64_t n_cells, int nloc, int64_t n_node,
                      const int32_t* degree, const int64_t* seeds, int64_t* order) {
  if (!cells || !degree || !seeds || !order || n_cells < 0 || nloc < 1 || n_node < 1)
    return sem::fail(SEM_E_INVALID, "sem_cuthill_mckee: invalid arguments");
  NodeCells nc;
  if (int rc = node_cells(cells, n_cells, nloc, n_node, nc)) return rc;
  std::vector<uint8_t> seen((size_t)n_node, 0);
  std::vector<uint32_t> fresh;
  int64_t N = 0;
  for (int64_t z = 0; z < n_node && N < n_node; ++z) {
    const int64_t seed = seeds[z];
    if (seed < 0 || seed >= n_node) return sem::fail(SEM_E_INVALID, "seed out of range");
    if (seen[(size_t)seed]) continue;
    seen[(size_t)seed] = 1;
    order[N++] = seed;
    int64_t lo = N - 1, hi = N;
    while (lo < hi) {
      for (int64_t ii = lo; ii < hi; ++ii) {
        const int64_t i = order[ii];
        fresh.clear();
        for (int64_t t = nc.ptr[(size_t)i]; t < nc.ptr[(size_t)i + 1]; ++t) {
          const uint32_t* c = cells + (int64_t)nc.cells[(size_t)t] * nloc;
          for (int k = 0; k < nloc; ++k)
            if (!seen[c[k]]) {
              seen[c[k]] = 1;
              fresh.push_back(c[k]);
            }
        }
        std::sort(fresh.begin(), fresh.end());
        std::stable_sort(fresh.begin(), fresh.end(),
                         [&](uint32_t a, uint32_t b) { return degree[a] < degree[b]; });
        for (uint32_t v : fresh) order[N++] = v;
      }
      lo = hi;
      hi = N;
    }
  }
  if (N != n_node) return sem::fail(SEM_E_INVALID, "sem_cuthill_mckee: seeds do not cover every node");
  return SEM_OK;
}

}  // extern "C"
