// In-memory adjacency: CSR rows in CPython-set iteration order plus the slot
// each entry occupies in its row's set table (needed when a row enters the
// frontier union as the adjacency set itself, models.py:282 `else to_neigh`).
#pragma once

#include <sys/mman.h>

#include <cstddef>
#include <cstdint>
#include <new>
#include <vector>

namespace gs {

// Allocator for the graph-sized arrays: anonymous mappings advised for
// transparent huge pages.  The sampler reads these arrays at random (a row
// per frontier node, hundreds of MB at the synthetic sizes); on 4-KiB pages
// nearly every such read also misses the TLB, and a software prefetch that
// misses the TLB is not guaranteed to be serviced.
template <class T>
struct HugeAlloc {
    using value_type = T;
    HugeAlloc() = default;
    template <class U>
    HugeAlloc(const HugeAlloc<U>&) {}
    T* allocate(size_t n) {
        const size_t bytes = n * sizeof(T);
        if (bytes < (size_t(2) << 20)) return static_cast<T*>(::operator new(bytes));
        void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
        if (p == MAP_FAILED) throw std::bad_alloc();
        (void)madvise(p, bytes, MADV_HUGEPAGE);
        return static_cast<T*>(p);
    }
    void deallocate(T* p, size_t n) {
        const size_t bytes = n * sizeof(T);
        if (bytes < (size_t(2) << 20)) ::operator delete(p);
        else munmap(p, bytes);
    }
    template <class U>
    bool operator==(const HugeAlloc<U>&) const { return true; }
    template <class U>
    bool operator!=(const HugeAlloc<U>&) const { return false; }
};
template <class T>
using hvec = std::vector<T, HugeAlloc<T>>;

struct Graph {
    int64_t n_nodes = 0;
    int64_t n_entries = 0;
    int64_t max_degree = 0;
    hvec<int64_t> row_ptr;          // [n_nodes + 1]
    hvec<int32_t> col;              // [n_entries]
    hvec<uint32_t> slot;            // [n_entries] slot in the row's set table
    hvec<uint8_t> log2size;         // [n_nodes]  table size = 1 << log2size
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
