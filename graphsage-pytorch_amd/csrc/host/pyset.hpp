// CPython 3.10 set restated for non-negative int keys (hash(i) == i), because
// the reference's frontier order IS a set's iteration order:
//   models.py:282  set(random.sample(...))        -> PySet::add per element
//   models.py:285  samp_neigh | set([node])        -> copy_of(...) + merge
//   models.py:286  list(set.union(*samp_neighs))   -> copy_of(first) + merge each
//   dataCenter.py:40-41 adj[p].add(q)              -> PySet::add (CSR builder)
// Rules follow Objects/setobject.c: LINEAR_PROBES = 9, PERTURB_SHIFT = 5,
// PySet_MINSIZE = 8, grow at fill*5 >= mask*3 to used*4 (used*2 above 50000),
// set_merge's pre-resize / slot-copy / insert_clean fast paths.  The reference
// never deletes from these sets, so there are no dummy entries (fill == used);
// a caller-built row with dummies is flagged by fill > used.
//
// Tables of up to kInline slots live inside the object (a sampled
// neighbourhood of k <= 25 never exceeds 128 slots), so the per-node sets of
// a hop are built without touching the heap.
#pragma once

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <vector>

namespace gs {

struct PySet {
    static constexpr int32_t EMPTY = -1;
    static constexpr size_t MINSIZE = 8;
    static constexpr size_t LINEAR_PROBES = 9;
    static constexpr int PERTURB_SHIFT = 5;
    static constexpr size_t kInline = 128;

    int32_t small_[kInline];
    std::vector<int32_t> big_;
    int32_t* tab = small_;
    size_t mask = MINSIZE - 1;
    int64_t fill = 0;
    int64_t used = 0;

    PySet() { std::fill_n(small_, MINSIZE, EMPTY); }
    PySet(const PySet& o) { *this = o; }
    PySet& operator=(const PySet& o) {
        if (this == &o) return *this;
        mask = o.mask;
        fill = o.fill;
        used = o.used;
        if (mask + 1 <= kInline) {
            std::memcpy(small_, o.tab, (mask + 1) * sizeof(int32_t));
            tab = small_;
        } else {
            big_.assign(o.tab, o.tab + mask + 1);
            tab = big_.data();
        }
        return *this;
    }

    void reset() {
        std::fill_n(small_, MINSIZE, EMPTY);
        tab = small_;
        mask = MINSIZE - 1;
        fill = used = 0;
    }

    size_t size() const { return mask + 1; }

    // Point `tab` at an EMPTY table of `n` slots (inline when it fits).
    void alloc_table(size_t n) {
        if (n <= kInline) {
            tab = small_;
        } else {
            big_.assign(n, EMPTY);
            tab = big_.data();
        }
        if (tab == small_) std::memset(small_, 0xFF, n * sizeof(int32_t));  // EMPTY == -1
        mask = n - 1;
    }

    // set_insert_clean: key known absent, table known to have room.
    static inline void insert_clean(int32_t* t, size_t m, int32_t key) {
        size_t perturb = static_cast<size_t>(key);
        size_t i = static_cast<size_t>(key) & m;
        for (;;) {
            int32_t* e = t + i;
            if (*e == EMPTY) {
                *e = key;
                return;
            }
            if (i + LINEAR_PROBES <= m) {
                for (size_t j = 0; j < LINEAR_PROBES; ++j) {
                    ++e;
                    if (*e == EMPTY) {
                        *e = key;
                        return;
                    }
                }
            }
            perturb >>= PERTURB_SHIFT;
            i = (i * 5 + 1 + perturb) & m;
        }
    }

    // set_table_resize: smallest power of two > minused, re-inserted in slot order.
    void resize(int64_t minused) {
        size_t newsize = MINSIZE;
        while (newsize <= static_cast<size_t>(minused)) newsize <<= 1;
        int32_t keep_small[kInline];
        std::vector<int32_t> keep_big;
        const int32_t* old;
        const size_t old_n = mask + 1;
        if (tab == small_) {
            std::memcpy(keep_small, small_, old_n * sizeof(int32_t));
            old = keep_small;
        } else {
            keep_big.swap(big_);
            old = keep_big.data();
        }
        alloc_table(newsize);
        for (size_t s = 0; s < old_n; ++s)
            if (old[s] != EMPTY) insert_clean(tab, mask, old[s]);
        fill = used;
    }

    // set_add_entry.  Returns true when the key was new.  The home slot is
    // settled without a data-dependent branch when it holds the key or is
    // empty (the common cases of a union, whose keys repeat often).
    bool add(int32_t key) {
        {
            const size_t i0 = static_cast<size_t>(key) & mask;
            const int32_t cur = tab[i0];
            if (cur == key || cur == EMPTY) {
                const bool fresh = cur == EMPTY;
                tab[i0] = key;
                fill += fresh;
                used += fresh;
                if (static_cast<size_t>(fill) * 5 >= mask * 3) resize(used > 50000 ? used * 2 : used * 4);
                return fresh;
            }
        }
        size_t perturb = static_cast<size_t>(key);
        size_t i = static_cast<size_t>(key) & mask;
        int32_t* e;
        for (;;) {
            e = tab + i;
            size_t probes = (i + LINEAR_PROBES <= mask) ? LINEAR_PROBES : 0;
            for (;;) {
                if (*e == EMPTY) goto found_unused;
                if (*e == key) return false;
                if (probes-- == 0) break;
                ++e;
            }
            perturb >>= PERTURB_SHIFT;
            i = (i * 5 + 1 + perturb) & mask;
        }
    found_unused:
        *e = key;
        ++fill;
        ++used;
        if (static_cast<size_t>(fill) * 5 < mask * 3) return true;
        resize(used > 50000 ? used * 2 : used * 4);
        return true;
    }

    // add() of a key known to be absent (set(random.sample(...)): distinct
    // sampled entries of one row): the same slot and resizes as add(), without
    // comparing against the keys on the probe path.
    void add_absent(int32_t key) {
        insert_clean(tab, mask, key);
        ++fill;
        ++used;
        if (static_cast<size_t>(fill) * 5 >= mask * 3) resize(used > 50000 ? used * 2 : used * 4);
    }

    // Slot of a present key (same probe walk as add), or -1.
    int64_t find_slot(int32_t key) const {
        size_t perturb = static_cast<size_t>(key);
        size_t i = static_cast<size_t>(key) & mask;
        for (;;) {
            const int32_t* e = tab + i;
            size_t probes = (i + LINEAR_PROBES <= mask) ? LINEAR_PROBES : 0;
            size_t s = i;
            for (;;) {
                if (*e == EMPTY) return -1;
                if (*e == key) return static_cast<int64_t>(s);
                if (probes-- == 0) break;
                ++e;
                ++s;
            }
            perturb >>= PERTURB_SHIFT;
            i = (i * 5 + 1 + perturb) & mask;
        }
    }

    // set_merge(this, other) where only other's iteration order and counts
    // matter (this non-empty): pre-resize, then set_add_entry per key.
    template <class K>
    void merge_items(const K* keys, int64_t n_used) {
        if (n_used == 0) return;
        if ((fill + n_used) * 5 >= static_cast<int64_t>(mask) * 3) resize((used + n_used) * 2);
        if (fill == 0) {  // cannot happen for the callers' non-empty targets
            fill = used = n_used;
            for (int64_t t = 0; t < n_used; ++t) insert_clean(tab, mask, keys[t]);
            return;
        }
        for (int64_t t = 0; t < n_used; ++t) add(keys[t]);
    }

    // merge_items over a run of key lists (set.union(first, *rest) after the
    // copy of the first), prefetching each key's home slot kAhead keys early:
    // the union table outgrows L1 and its probes are otherwise serial misses.
    template <class K>
    void merge_runs(const K* keys, const int32_t* ptr, int64_t n_runs) {
        constexpr int64_t kAhead = 16;
        const int64_t total = ptr[n_runs] - ptr[0];
        const K* base = keys + ptr[0];
        int64_t t = 0;
        for (int64_t r = 0; r < n_runs; ++r) {
            const int64_t n_used = ptr[r + 1] - ptr[r];
            if (n_used == 0) continue;
            if ((fill + n_used) * 5 >= static_cast<int64_t>(mask) * 3) resize((used + n_used) * 2);
            for (int64_t e = t + n_used; t < e; ++t) {
                if (t + kAhead < total) __builtin_prefetch(tab + (static_cast<size_t>(base[t + kAhead]) & mask));
                add(base[t]);
            }
        }
    }

    // set_merge(this, other).
    void merge(const PySet& o) {
        if (&o == this || o.used == 0) return;
        if ((fill + o.used) * 5 >= static_cast<int64_t>(mask) * 3) resize((used + o.used) * 2);
        if (fill == 0 && mask == o.mask && o.fill == o.used) {
            std::memcpy(tab, o.tab, (mask + 1) * sizeof(int32_t));
            fill = o.fill;
            used = o.used;
            return;
        }
        if (fill == 0) {
            fill = used = o.used;
            for (size_t s = 0; s <= o.mask; ++s)
                if (o.tab[s] != EMPTY) insert_clean(tab, mask, o.tab[s]);
            return;
        }
        for (size_t s = 0; s <= o.mask; ++s)
            if (o.tab[s] != EMPTY) add(o.tab[s]);
    }

    // set_merge with a one-element set {key} (the `| set([node])` of :285):
    // {key} has mask 7, used 1, key in slot key & 7.
    void merge_single(int32_t key) {
        if ((fill + 1) * 5 >= static_cast<int64_t>(mask) * 3) resize((used + 1) * 2);
        if (fill == 0 && mask == MINSIZE - 1) {  // slot copy of {key}
            std::fill_n(tab, MINSIZE, EMPTY);
            tab[static_cast<size_t>(key) & 7] = key;
            fill = used = 1;
            return;
        }
        if (fill == 0) {
            fill = used = 1;
            insert_clean(tab, mask, key);
            return;
        }
        add(key);
    }

    // copy_into(*this, o) for o = a set whose table is given verbatim (an
    // adjacency row's own layout: keys in slot order, `slots` their slots in
    // a table of m0 + 1), without building o: the copy's table is sized from
    // o.used alone, then takes o's slots verbatim when the sizes agree and o
    // has no dummies (set_merge's slot-copy path), else insert_clean in o's
    // slot order.
    void assign_copy_of_layout(size_t m0, const int32_t* keys, const uint32_t* slots, int64_t n, bool dummies) {
        size_t newsize = MINSIZE;
        if (n * 5 >= static_cast<int64_t>(MINSIZE - 1) * 3)
            while (newsize <= static_cast<size_t>(2 * n)) newsize <<= 1;
        alloc_table(newsize);
        fill = used = n;
        if (mask == m0 && !dummies) {
            for (int64_t t = 0; t < n; ++t) tab[slots[t]] = keys[t];
        } else {
            for (int64_t t = 0; t < n; ++t) insert_clean(tab, mask, keys[t]);
        }
    }

    // A set whose table is given verbatim (an adjacency row's own layout).
    void assign_layout(size_t m, const int32_t* keys, const uint32_t* slots, int64_t n) {
        alloc_table(m + 1);
        for (int64_t t = 0; t < n; ++t) tab[slots[t]] = keys[t];
        fill = used = n;
    }

    template <class F>
    void for_each(F&& f) const {
        for (size_t s = 0; s <= mask; ++s)
            if (tab[s] != EMPTY) f(tab[s]);
    }
};

// set.copy() / make_new_set(iterable=set): an empty set merged with `o`.
inline void copy_into(PySet& r, const PySet& o) {
    r.reset();
    r.merge(o);
}

inline PySet copy_of(const PySet& o) {
    PySet r;
    r.merge(o);
    return r;
}

}  // namespace gs
