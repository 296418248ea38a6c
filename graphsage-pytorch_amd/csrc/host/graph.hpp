// In-memory adjacency: CSR rows in CPython-set iteration order plus the slot
// each entry occupies in its row's set table (needed when a row enters the
// frontier union as the adjacency set itself, models.py:282 `else to_neigh`).
#pragma once

#include <cstdint>
#include <vector>

namespace gs {

struct Graph {
    int64_t n_nodes = 0;
    int64_t n_entries = 0;
    int64_t max_degree = 0;
    std::vector<int64_t> row_ptr;   // [n_nodes + 1]
    std::vector<int32_t> col;       // [n_entries]
    std::vector<uint32_t> slot;     // [n_entries] slot in the row's set table
    std::vector<uint8_t> log2size;  // [n_nodes]  table size = 1 << log2size
    std::vector<uint8_t> dirty;     // [n_nodes] or empty: row set holds dummy entries
    int64_t degree(int64_t v) const { return row_ptr[v + 1] - row_ptr[v]; }
};

Graph* build_graph(const int64_t* src, const int64_t* dst, int64_t n_pairs, int64_t n_nodes,
                   int32_t n_threads);
Graph* graph_from_tables(int64_t n_nodes, const int64_t* row_ptr, const int32_t* col,
                         const uint32_t* slot, const uint8_t* log2size, const uint8_t* dirty);
int64_t rmat_pairs(int32_t scale, int64_t n_pairs, double a, double b, double c, uint64_t seed,
                   int32_t permute, int32_t n_threads, int64_t* src, int64_t* dst);

}  // namespace gs
