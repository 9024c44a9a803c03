// Any-hit BVH for shadow rays (host build; device walk: rtg_common.hpp walk_wide_any).
#pragma once
#include <hip/hip_runtime.h>

#include <vector>

#include "rtg_device.hpp"

namespace rtg {

// Topology of the any-hit tree (RTG_AHB environment variable):
//   AHB_EXACT (default) binned-SAH 4-wide tree over the reference's leaves: every cull box a
//             reference leaf box, so culling is exact; large-leaf scenes keep the cooperative
//             reference walk for their shadow rays (a lane alone in a 255-face pole fan stalls
//             its wave);
//   AHB_SPLIT (opt-in) the same, the faces of large leaves split into their own primitives
//             with padded triangle boxes (exact for rays more than ~1 degree off a face's
//             plane; rtg_ahb.cpp), and large-leaf scenes take the tree;
//   AHB_REF   the reference's own BVH collapsed to 4 wide (round 2's tree, A/B).
enum AhbMode { AHB_REF = 0, AHB_EXACT = 1, AHB_SPLIT = 2 };

struct AhbStats {
    long long leaf_prims = 0;       // reference leaves taken whole (exact box)
    long long face_prims = 0;       // single faces of large leaves (padded triangle box)
    long long exact_faces = 0;      // of those, ill-conditioned faces kept on their leaf box
    long long nodes = 0, entries = 0;
    int max_depth = 0;
};

// Builds the any-hit tree of one mesh: `nodes` / `ext` are the uploaded pre-order reference
// records (rtg_device.hpp), [node_begin, node_end) the mesh's range, `tris` the BVH-ordered
// face records {v0}, {v0 - v1}, {v0 - v2}.  `reach` bounds |coordinate| of any shadow-ray
// origin or end point in the mesh's local space (the padding of split faces scales with it).
// Appends wide nodes to `out` and face entries (a copy of the face record, the reference leaf
// node's index in the first record's w) to `entries`; returns the root's index in `out`.
int build_ahb(const std::vector<float4>& nodes, const std::vector<int2>& ext, int node_begin, int node_end,
              const float4* tris, double reach, AhbMode mode, std::vector<WNode>& out, std::vector<float4>& entries,
              AhbStats* st);

// Structural check (CPU tests): coverage of the mesh's faces, reference leaves, box nesting
// and containment of every entry's triangle.  Returns the number of violations.
long long ahb_validate(const std::vector<WNode>& out, const std::vector<float4>& entries, int root,
                       const std::vector<float4>& nodes, const std::vector<int2>& ext, int node_begin, int node_end,
                       const float4* tris);

}  // namespace rtg
