// Device half of extend_nodes' negatives (kernels/unsup_ball.hip), called by
// host/unsup.cpp when a gs_unsup has a device attached.  Plain C++ (no HIP
// types): the host translation units are built without the HIP headers.
#pragma once

#include <cstdint>
#include <vector>

namespace gs {

struct Graph;
struct UnsupDev;

UnsupDev* unsup_dev_create(const Graph& g, const std::vector<int32_t>& copy_order,
                           const std::vector<int32_t>& set_order, void* stream);
void unsup_dev_destroy(UnsupDev* d);
// The n_walk_len-hop balls of nodes[0..n) (models.py:154-162): len(neighbors)
// and |set(train) ∩ neighbors| per node; also prepares the far-list picks.
void unsup_dev_balls(UnsupDev* d, const int64_t* nodes, int n, int hops, int64_t* ball_size, int64_t* train_in_ball);
// out[q] = element req_j[q] of node req_r[q]'s far list in order req_kind[q]
// (0: set(train).copy() order, 1: ascending ids, 2: set(train) order), ball
// members skipped.
void unsup_dev_select(UnsupDev* d, const std::vector<int32_t>& req_r, const std::vector<int32_t>& req_j,
                      const std::vector<uint8_t>& req_kind, std::vector<int32_t>& out);

// The whole far lists of balls[q] in set(train) order, concatenated at
// base[q] (base has balls.size() + 1 entries).
void unsup_dev_far_lists(UnsupDev* d, const std::vector<int32_t>& balls, const std::vector<int64_t>& base,
                         std::vector<int32_t>& out);

}  // namespace gs
