// Any-hit BVH for shadow rays (rtg_ahb.hpp): host build.
//
// CastShadowRay (raytracer.cpp:585-623) answers a boolean, so its traversal structure is free;
// what must stay the reference's are the decisions (rtg_common.hpp walk_wide_any): a face f of
// reference leaf L decides "shadow" when IntersectFace accepts it below the light distance and
// L's box B_L passes the slab test at that distance, and only a face that IntersectFace accepts
// and whose B_L passes at the initial minT can matter at all.  The tree below is therefore
// built for speed, and its only obligation is to reach every face that can matter: a subtree
// may be culled only when its box, conservatively tested at the initial minT, proves that.
// Each primitive carries a cull box that does:
//   * a whole reference leaf with at most kSplitLeaf faces: B_L itself, copied bit for bit --
//     a face whose B_L fails at minT0 cannot matter, and every node box contains B_L (exact
//     float min / max), so the slab test (monotone in the box) culls exactly;
//   * a single face of a larger leaf (the reference's midpoint split leaves pole fans of
//     65-255 faces): its triangle's box, padded.  IntersectFace accepts f only where the ray
//     passes the triangle up to the rounding of Cramer's rule: the computed beta, gamma, t
//     differ from the exact ones by ~ 5 u |A - o| / (sin(alpha) sin(theta)) in position
//     (u = 2^-24, alpha the triangle's angle at v0, theta the ray's angle to its plane), and
//     |A - o| <= `reach`.  The pad 2^p kappa reach (kappa = |E1||E2| / |E1 x E2| =
//     1 / sin(alpha); p = pad_exp(), -16 as shipped) covers that for every ray with
//     sin(theta) >= 5 u 2^-p = 5 * 2^-8, i.e. more than 1.1 degrees off the face's plane
//     (2.2 degrees with a factor-2 margin on the estimate; p = -12 would give 0.07 / 0.14);
//     a face with kappa > 64 (a sliver) keeps B_L as its cull box instead;
// so the walk's answer equals the reference's up to rays that graze a face of a large leaf
// within ~1-2 degrees and are accepted by rounding alone.  That is why the split tree is
// opt-in (RTG_AHB=split) and the default tree keeps every reference leaf whole (DESIGN.md §2;
// both tested against the reference walk, RTG_RENDER_EXACT_SHADOW, image for image).
#include "rtg_ahb.hpp"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>

namespace rtg {
namespace {

constexpr int kSplitLeaf = 8;          // reference leaves above this many faces are split into faces
constexpr int kMaxLeafFaces = 8;
constexpr int kBins = 32;
// Leaf shape: a range of at most `leaf_faces` faces is a leaf outright; up to kMaxLeafFaces
// the SAH decides, with a face test costing `isect_cost` box tests (RTG_AHB_LEAF /
// RTG_AHB_CI: A/B experiments).
int env_int(const char* name, int dflt) {
    const char* v = std::getenv(name);
    return v ? std::atoi(v) : dflt;
}
int leaf_faces() { return env_int("RTG_AHB_LEAF", 2); }
// pad of a split face = 2^pad_exp kappa reach (RTG_AHB_PADEXP: A/B experiments)
int pad_exp() { return env_int("RTG_AHB_PADEXP", -16); }
// split faces with kappa above this keep their leaf box (RTG_AHB_KAPPA: A/B experiments)
double kappa_max() { return env_int("RTG_AHB_KAPPA", 64); }
double isect_cost() {
    const char* v = std::getenv("RTG_AHB_CI");
    return v ? std::atof(v) : 2.0;
}

struct Prim {
    float lo[3], hi[3];
    float c[3];                        // centroid (binning)
    int first, count;                  // faces [first, first + count), BVH order
    int ref;                           // reference leaf node (global index)
};

struct BNode {
    float lo[3], hi[3];
    int left = -1, right = -1;         // inner: children; leaf: left < 0
    int pbeg = 0, pcnt = 0;            // leaf: prims [pbeg, pbeg + pcnt)
    int faces = 0;
};

int leaf_of(const std::vector<float4>& nodes, int i) {
    int l;
    std::memcpy(&l, &nodes[2 * i + 1].w, 4);
    return l;
}
int skip_of(const std::vector<float4>& nodes, int i) {
    int k;
    std::memcpy(&k, &nodes[2 * i + 1].z, 4);
    return k;
}
void box_of(const std::vector<float4>& nodes, int i, float* lo, float* hi) {
    const float4 a = nodes[2 * i], b = nodes[2 * i + 1];
    lo[0] = a.x; lo[1] = a.y; lo[2] = a.z;
    hi[0] = a.w; hi[1] = b.x; hi[2] = b.y;
}
void leaf_range(const std::vector<float4>& nodes, const std::vector<int2>& ext, int i, int& first, int& count) {
    const int l = leaf_of(nodes, i);
    if (l == LEAF_EXT) { first = ext[i].x; count = ext[i].y; }
    else { first = l >> 8; count = l & 255; }
}
float down(double v) {
    float f = (float)v;
    if ((double)f > v) f = std::nextafter(f, -INFINITY);
    return f;
}
float up(double v) {
    float f = (float)v;
    if ((double)f < v) f = std::nextafter(f, INFINITY);
    return f;
}
double area(const float* lo, const float* hi) {
    const double dx = (double)hi[0] - lo[0], dy = (double)hi[1] - lo[1], dz = (double)hi[2] - lo[2];
    if (!(dx >= 0 && dy >= 0 && dz >= 0)) return 0.0;
    return dx * dy + dy * dz + dz * dx;
}
void grow(float* lo, float* hi, const float* l2, const float* h2) {
    for (int a = 0; a < 3; ++a) { lo[a] = std::min(lo[a], l2[a]); hi[a] = std::max(hi[a], h2[a]); }
}
void set_empty(float* lo, float* hi) {
    for (int a = 0; a < 3; ++a) { lo[a] = INFINITY; hi[a] = -INFINITY; }
}

struct Builder {
    std::vector<Prim>& P;
    std::vector<BNode> N;
    explicit Builder(std::vector<Prim>& p) : P(p) {}

    int make_leaf(int b, int e) {
        BNode n;
        set_empty(n.lo, n.hi);
        for (int i = b; i < e; ++i) { grow(n.lo, n.hi, P[i].lo, P[i].hi); n.faces += P[i].count; }
        n.pbeg = b;
        n.pcnt = e - b;
        N.push_back(n);
        return (int)N.size() - 1;
    }
    int make_inner(int l, int r) {
        BNode n;
        std::memcpy(n.lo, N[l].lo, sizeof n.lo);
        std::memcpy(n.hi, N[l].hi, sizeof n.hi);
        grow(n.lo, n.hi, N[r].lo, N[r].hi);
        n.left = l;
        n.right = r;
        n.faces = N[l].faces + N[r].faces;
        N.push_back(n);
        return (int)N.size() - 1;
    }

    // binned SAH over prims [b, e); recursion depth is O(log n) for the SAH splits and bounded
    // by the median fall-back otherwise
    int build(int b, int e) {
        int faces = 0;
        float lo[3], hi[3], clo[3], chi[3];
        set_empty(lo, hi);
        set_empty(clo, chi);
        for (int i = b; i < e; ++i) {
            faces += P[i].count;
            grow(lo, hi, P[i].lo, P[i].hi);
            grow(clo, chi, P[i].c, P[i].c);
        }
        if (e - b == 1 || faces <= leaf_faces()) {
            if (faces <= 255) return make_leaf(b, e);
        }
        int axis = 0;
        for (int a = 1; a < 3; ++a)
            if ((double)chi[a] - clo[a] > (double)chi[axis] - clo[axis]) axis = a;
        const double ext = (double)chi[axis] - clo[axis];
        int mid = -1;
        if (ext > 0) {
            float blo[kBins][3], bhi[kBins][3];
            int bcnt[kBins] = {0};
            for (int k = 0; k < kBins; ++k) set_empty(blo[k], bhi[k]);
            auto bin = [&](const Prim& p) {
                int k = (int)(((double)p.c[axis] - clo[axis]) / ext * kBins);
                return std::min(kBins - 1, std::max(0, k));
            };
            for (int i = b; i < e; ++i) {
                const int k = bin(P[i]);
                bcnt[k] += P[i].count;
                grow(blo[k], bhi[k], P[i].lo, P[i].hi);
            }
            // sweep: cost(split after bin k) = A_L N_L + A_R N_R
            double rarea[kBins];
            int rcnt[kBins];
            float rl[3], rh[3];
            set_empty(rl, rh);
            int rc = 0;
            for (int k = kBins - 1; k > 0; --k) {
                grow(rl, rh, blo[k], bhi[k]);
                rc += bcnt[k];
                rarea[k] = area(rl, rh);
                rcnt[k] = rc;
            }
            float ll[3], lh[3];
            set_empty(ll, lh);
            int lc = 0;
            double best = INFINITY;
            int bestk = -1;
            for (int k = 0; k < kBins - 1; ++k) {
                grow(ll, lh, blo[k], bhi[k]);
                lc += bcnt[k];
                if (lc == 0 || rcnt[k + 1] == 0) continue;
                const double cost = area(ll, lh) * lc + rarea[k + 1] * rcnt[k + 1];
                if (cost < best) { best = cost; bestk = k; }
            }
            // SAH (relative to this node's area): leaf = A N c_i, split = A + (A_L N_L + A_R N_R) c_i
            const double ci = isect_cost();
            if (faces <= kMaxLeafFaces && area(lo, hi) + best * ci >= area(lo, hi) * faces * ci) return make_leaf(b, e);
            if (bestk >= 0) {
                Prim* pm = std::partition(P.data() + b, P.data() + e, [&](const Prim& p) { return bin(p) <= bestk; });
                mid = (int)(pm - P.data());
                if (mid == b || mid == e) mid = -1;
            }
        }
        if (mid < 0) {
            // no spatial split: a leaf if it fits, else halve by count
            if (faces <= kMaxLeafFaces) return make_leaf(b, e);
            mid = (b + e) / 2;
        }
        const int l = build(b, mid);
        const int r = build(mid, e);
        return make_inner(l, r);
    }

    // the reference's own topology over the same prims (AHB_REF): prims are the reference's
    // leaves in pre-order, so a subtree is a contiguous prim range
    int from_reference(const std::vector<float4>& nodes, int i, int& pcur, const std::vector<int>& chunks) {
        if (leaf_of(nodes, i) >= 0) {
            const int b = pcur, e = pcur + chunks[i];
            pcur = e;
            return chunk_tree(b, e);
        }
        const int l = from_reference(nodes, i + 1, pcur, chunks);
        const int r = from_reference(nodes, skip_of(nodes, i + 1), pcur, chunks);
        return make_inner(l, r);
    }
    int chunk_tree(int b, int e) {   // a leaf split into <= 255-face chunks
        if (e - b == 1) return make_leaf(b, e);
        const int m = (b + e) / 2;
        const int l = chunk_tree(b, m);
        const int r = chunk_tree(m, e);
        return make_inner(l, r);
    }
};

}  // namespace

int build_ahb(const std::vector<float4>& nodes, const std::vector<int2>& ext, int node_begin, int node_end,
              const float4* tris, double reach, AhbMode mode, std::vector<WNode>& out, std::vector<float4>& entries,
              AhbStats* st) {
    if (node_end <= node_begin) return -1;
    std::vector<Prim> P;
    std::vector<int> chunks(nodes.size() / 2, 0);   // AHB_REF: prims per reference leaf
    const double u = std::ldexp(1.0, pad_exp());
    const double kmax = kappa_max();
    for (int i = node_begin; i < node_end; ++i) {
        if (leaf_of(nodes, i) < 0) continue;
        int first, count;
        leaf_range(nodes, ext, i, first, count);
        Prim leafp;
        box_of(nodes, i, leafp.lo, leafp.hi);
        for (int a = 0; a < 3; ++a) leafp.c[a] = (float)(0.5 * ((double)leafp.lo[a] + leafp.hi[a]));
        leafp.ref = i;
        if (mode != AHB_SPLIT || count <= kSplitLeaf) {
            for (int f = first; f < first + count; f += 255) {   // entry ranges hold <= 255 faces
                Prim p = leafp;
                p.first = f;
                p.count = std::min(255, first + count - f);
                P.push_back(p);
                ++chunks[i];
            }
            if (st) ++st->leaf_prims;
            continue;
        }
        for (int f = first; f < first + count; ++f) {
            Prim p = leafp;
            p.first = f;
            p.count = 1;
            const float4 A = tris[3 * (size_t)f], E1 = tris[3 * (size_t)f + 1], E2 = tris[3 * (size_t)f + 2];
            const double a[3] = {A.x, A.y, A.z}, e1[3] = {E1.x, E1.y, E1.z}, e2[3] = {E2.x, E2.y, E2.z};
            const double cx = e1[1] * e2[2] - e1[2] * e2[1], cy = e1[2] * e2[0] - e1[0] * e2[2],
                         cz = e1[0] * e2[1] - e1[1] * e2[0];
            const double n1 = std::sqrt(e1[0] * e1[0] + e1[1] * e1[1] + e1[2] * e1[2]);
            const double n2 = std::sqrt(e2[0] * e2[0] + e2[1] * e2[1] + e2[2] * e2[2]);
            const double nc = std::sqrt(cx * cx + cy * cy + cz * cz);
            const double kappa = nc > 0 ? n1 * n2 / nc : INFINITY;
            if (!(kappa <= kmax)) {
                if (st) ++st->exact_faces;           // a sliver: its leaf box
            } else {
                double mag = 0;
                for (int k = 0; k < 3; ++k)
                    mag = std::max({mag, std::fabs(a[k]), std::fabs(a[k] - e1[k]), std::fabs(a[k] - e2[k])});
                const double pad = u * kappa * reach + std::ldexp(mag, -20);
                for (int k = 0; k < 3; ++k) {
                    // the exact-arithmetic triangle A - beta E1 - gamma E2
                    const double v0 = a[k], v1 = a[k] - e1[k], v2 = a[k] - e2[k];
                    p.lo[k] = down(std::min({v0, v1, v2}) - pad);
                    p.hi[k] = up(std::max({v0, v1, v2}) + pad);
                    p.c[k] = (float)((v0 + v1 + v2) / 3.0);
                }
            }
            P.push_back(p);
            if (st) ++st->face_prims;
        }
    }
    if (P.empty()) return -1;
    Builder B(P);
    int root;
    if (mode == AHB_REF) {
        int pcur = 0;
        root = B.from_reference(nodes, node_begin, pcur, chunks);
    } else {
        root = B.build(0, (int)P.size());
    }
    // collapse to 4 wide (open the inner child of largest surface area until four remain),
    // emitting each leaf's faces as entries in depth-first order
    struct Job { int bn, owner, slot, depth; };
    std::vector<Job> jobs{{root, -1, 0, 1}};
    int rootIdx = -1;
    while (!jobs.empty()) {
        const Job j = jobs.back();
        jobs.pop_back();
        std::vector<int> C;
        if (B.N[j.bn].left < 0) C.push_back(j.bn);
        else { C.push_back(B.N[j.bn].left); C.push_back(B.N[j.bn].right); }
        while (C.size() < 4) {
            int best = -1;
            double ba = -1.0;
            for (size_t k = 0; k < C.size(); ++k)
                if (B.N[C[k]].left >= 0 && area(B.N[C[k]].lo, B.N[C[k]].hi) > ba) {
                    ba = area(B.N[C[k]].lo, B.N[C[k]].hi);
                    best = (int)k;
                }
            if (best < 0) break;
            const int x = C[best];
            C[best] = B.N[x].left;
            C.insert(C.begin() + best + 1, B.N[x].right);
        }
        const int w = (int)out.size();
        out.emplace_back();
        if (st) { ++st->nodes; st->max_depth = std::max(st->max_depth, j.depth); }
        float* lo[3] = {&out[w].lox.x, &out[w].loy.x, &out[w].loz.x};
        float* hi[3] = {&out[w].hix.x, &out[w].hiy.x, &out[w].hiz.x};
        int* ch = &out[w].child.x;
        int* lf = &out[w].leaf.x;
        for (int k = 0; k < 4; ++k) {
            if (k >= (int)C.size()) {
                for (int a = 0; a < 3; ++a) { lo[a][k] = INFINITY; hi[a][k] = -INFINITY; }
                ch[k] = WCHILD_EMPTY;
                lf[k] = 0;
                continue;
            }
            const BNode& n = B.N[C[k]];
            for (int a = 0; a < 3; ++a) { lo[a][k] = n.lo[a]; hi[a][k] = n.hi[a]; }
            if (n.left >= 0) {
                ch[k] = WCHILD_EMPTY;      // set when the child node is emitted
                lf[k] = 0;
                continue;
            }
            const size_t e0 = entries.size() / 3;
            for (int q = n.pbeg; q < n.pbeg + n.pcnt; ++q)
                for (int f = P[q].first; f < P[q].first + P[q].count; ++f) {
                    // [0].w: the face's reference leaf node; [1].w: the face itself (global
                    // BVH-order index: the closest-hit walk reports it and orders ties by it)
                    float4 A = tris[3 * (size_t)f], E1 = tris[3 * (size_t)f + 1];
                    std::memcpy(&A.w, &P[q].ref, 4);
                    std::memcpy(&E1.w, &f, 4);
                    entries.push_back(A);
                    entries.push_back(E1);
                    entries.push_back(tris[3 * (size_t)f + 2]);
                }
            const size_t cnt = entries.size() / 3 - e0;
            if (e0 >= (1u << 23) || cnt > 255) return -2;   // entry index / count out of the leaf encoding
            ch[k] = -2;
            lf[k] = (int)((e0 << 8) | cnt);
            if (st) st->entries += (long long)cnt;
        }
        if (j.owner >= 0) (&out[j.owner].child.x)[j.slot] = w;
        else rootIdx = w;
        for (int k = (int)C.size() - 1; k >= 0; --k)
            if (B.N[C[k]].left >= 0) jobs.push_back({C[k], w, k, j.depth + 1});
    }
    return rootIdx;
}

}  // namespace rtg

namespace rtg {

// Structural check of one mesh's any-hit tree (CPU tests, rtg_desc_anyhit_check): every face
// of the mesh's node range appears in exactly one leaf entry (compared by its record's bits),
// each entry names a reference leaf that holds that face, every node's child boxes lie inside
// the box its parent slot gave it, and every entry's triangle (A, A - E1, A - E2 in exact
// arithmetic, to 2^-20 relative) lies inside its leaf slot's box.  Returns the violations.
long long ahb_validate(const std::vector<WNode>& out, const std::vector<float4>& entries, int root,
                       const std::vector<float4>& nodes, const std::vector<int2>& ext, int node_begin, int node_end,
                       const float4* tris) {
    auto key = [](const float4* r) {
        unsigned long long h = 1469598103934665603ull;
        const float v[9] = {r[0].x, r[0].y, r[0].z, r[1].x, r[1].y, r[1].z, r[2].x, r[2].y, r[2].z};
        for (float x : v) {
            unsigned u;
            std::memcpy(&u, &x, 4);
            h = (h ^ u) * 1099511628211ull;
        }
        return h;
    };
    std::vector<std::pair<unsigned long long, int>> want, got;
    for (int i = node_begin; i < node_end; ++i) {
        if (leaf_of(nodes, i) < 0) continue;
        int first, count;
        leaf_range(nodes, ext, i, first, count);
        for (int f = first; f < first + count; ++f) want.push_back({key(tris + 3 * (size_t)f), i});
    }
    long long bad = 0;
    if (root < 0) return want.empty() ? 0 : (long long)want.size();
    struct Item { int node; float lo[3], hi[3]; };
    std::vector<Item> st{{root, {-INFINITY, -INFINITY, -INFINITY}, {INFINITY, INFINITY, INFINITY}}};
    while (!st.empty()) {
        const Item it = st.back();
        st.pop_back();
        const WNode& W = out[it.node];
        const float* lo[3] = {&W.lox.x, &W.loy.x, &W.loz.x};
        const float* hi[3] = {&W.hix.x, &W.hiy.x, &W.hiz.x};
        for (int k = 0; k < 4; ++k) {
            const int c = (&W.child.x)[k];
            if (c == WCHILD_EMPTY) continue;
            float clo[3], chi[3];
            for (int a = 0; a < 3; ++a) {
                clo[a] = lo[a][k];
                chi[a] = hi[a][k];
                if (clo[a] < it.lo[a] || chi[a] > it.hi[a]) ++bad;
            }
            if (c >= 0) {
                Item n{c, {clo[0], clo[1], clo[2]}, {chi[0], chi[1], chi[2]}};
                st.push_back(n);
                continue;
            }
            const int lf = (&W.leaf.x)[k];
            for (int e = lf >> 8; e < (lf >> 8) + (lf & 255); ++e) {
                const float4* r = entries.data() + 3 * (size_t)e;
                int ref;
                std::memcpy(&ref, &r[0].w, 4);
                float4 rr[3] = {r[0], r[1], r[2]};
                rr[0].w = 0.f;
                got.push_back({key(rr), ref});
                if (ref < node_begin || ref >= node_end || leaf_of(nodes, ref) < 0) { ++bad; continue; }
                int face, lfirst, lcount;
                std::memcpy(&face, &r[1].w, 4);
                leaf_range(nodes, ext, ref, lfirst, lcount);
                // the named face is one of its reference leaf's, with this record
                if (face < lfirst || face >= lfirst + lcount || key(tris + 3 * (size_t)face) != key(rr)) ++bad;
                const double A[3] = {r[0].x, r[0].y, r[0].z}, E1[3] = {r[1].x, r[1].y, r[1].z},
                             E2[3] = {r[2].x, r[2].y, r[2].z};
                for (int a = 0; a < 3; ++a) {
                    // A - E1 is v1 up to the rounding of E1 = v0 - v1 (its magnitude's ulp)
                    const double tol = std::ldexp(std::max({std::fabs(A[a]), std::fabs(E1[a]), std::fabs(E2[a])}), -20);
                    for (const double v : {A[a], A[a] - E1[a], A[a] - E2[a]})
                        if (v < (double)clo[a] - tol || v > (double)chi[a] + tol) ++bad;
                }
            }
        }
    }
    std::sort(want.begin(), want.end());
    std::sort(got.begin(), got.end());
    if (want != got) bad += 1 + (long long)std::abs((long long)want.size() - (long long)got.size());
    return bad;
}

}  // namespace rtg
