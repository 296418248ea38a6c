// CPython 3.10 set restated for non-negative int keys (hash(i) == i), because
// the reference's frontier order IS a set's iteration order:
//   models.py:282  set(random.sample(...))        -> PySet::add per element
//   models.py:285  samp_neigh | set([node])        -> copy_of(...) + merge
//   models.py:286  list(set.union(*samp_neighs))   -> copy_of(first) + merge each
//   dataCenter.py:40-41 adj[p].add(q)              -> PySet::add (CSR builder)
// Rules follow Objects/setobject.c: LINEAR_PROBES = 9, PERTURB_SHIFT = 5,
// PySet_MINSIZE = 8, grow at fill*5 >= mask*3 to used*4 (used*2 above 50000),
// set_merge's pre-resize / slot-copy / insert_clean fast paths.  The reference
// never deletes from these sets, so there are no dummy entries (fill == used).
#pragma once

#include <cstdint>
#include <cstring>
#include <vector>

namespace gs {

struct PySet {
    static constexpr int64_t EMPTY = -1;
    static constexpr size_t MINSIZE = 8;
    static constexpr size_t LINEAR_PROBES = 9;
    static constexpr int PERTURB_SHIFT = 5;

    std::vector<int64_t> tab;
    size_t mask = MINSIZE - 1;
    int64_t fill = 0;
    int64_t used = 0;

    PySet() : tab(MINSIZE, EMPTY) {}

    void reset() {
        tab.assign(MINSIZE, EMPTY);
        mask = MINSIZE - 1;
        fill = used = 0;
    }

    // set_insert_clean: key known absent, table known to have room.
    static inline void insert_clean(int64_t* t, size_t m, int64_t key) {
        size_t perturb = static_cast<size_t>(key);
        size_t i = static_cast<size_t>(key) & m;
        for (;;) {
            int64_t* e = t + i;
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
        std::vector<int64_t> old;
        old.swap(tab);
        tab.assign(newsize, EMPTY);
        mask = newsize - 1;
        for (int64_t k : old)
            if (k != EMPTY) insert_clean(tab.data(), mask, k);
        fill = used;
    }

    // set_add_entry.  Returns true when the key was new.
    bool add(int64_t key) {
        size_t perturb = static_cast<size_t>(key);
        size_t i = static_cast<size_t>(key) & mask;
        int64_t* e;
        for (;;) {
            e = tab.data() + i;
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

    // Slot of a present key (same probe walk as add), or -1.
    int64_t find_slot(int64_t key) const {
        size_t perturb = static_cast<size_t>(key);
        size_t i = static_cast<size_t>(key) & mask;
        for (;;) {
            const int64_t* e = tab.data() + i;
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

    // set_merge(this, other).
    void merge(const PySet& o) {
        if (&o == this || o.used == 0) return;
        if ((fill + o.used) * 5 >= static_cast<int64_t>(mask) * 3) resize((used + o.used) * 2);
        if (fill == 0 && mask == o.mask && o.fill == o.used) {
            tab = o.tab;
            fill = o.fill;
            used = o.used;
            return;
        }
        if (fill == 0) {
            fill = used = o.used;
            for (int64_t k : o.tab)
                if (k != EMPTY) insert_clean(tab.data(), mask, k);
            return;
        }
        for (int64_t k : o.tab)
            if (k != EMPTY) add(k);
    }

    // set_merge with a one-element set {key} (the `| set([node])` of :285).
    void merge_single(int64_t key) {
        PySet one;
        one.add(key);
        merge(one);
    }

    // A set whose table is given verbatim (an adjacency row's own layout).
    void assign_layout(size_t m, const int64_t* keys, const uint32_t* slots, int64_t n) {
        tab.assign(m + 1, EMPTY);
        mask = m;
        for (int64_t t = 0; t < n; ++t) tab[slots[t]] = keys[t];
        fill = used = n;
    }

    template <class F>
    void for_each(F&& f) const {
        for (int64_t k : tab)
            if (k != EMPTY) f(k);
    }
};

// set.copy() / make_new_set(iterable=set): an empty set merged with `o`.
inline PySet copy_of(const PySet& o) {
    PySet r;
    r.merge(o);
    return r;
}

// Final mask of a set grown by `n` distinct adds from empty (no deletions):
// resizes depend only on the count of distinct keys.
inline size_t grown_mask(int64_t n) {
    size_t mask = PySet::MINSIZE - 1;
    int64_t fill = 0;
    for (int64_t u = 1; u <= n; ++u) {
        fill = u;
        if (static_cast<size_t>(fill) * 5 >= mask * 3) {
            const int64_t minused = u > 50000 ? u * 2 : u * 4;
            size_t ns = PySet::MINSIZE;
            while (ns <= static_cast<size_t>(minused)) ns <<= 1;
            mask = ns - 1;
        }
    }
    return mask;
}

}  // namespace gs
