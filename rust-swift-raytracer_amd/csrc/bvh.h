// bvh.h -- exact-pruning sphere BVH (host build, device layout).
//
// The reference tests every sphere in file order with a shrinking t_max
// (common.rs:241-247).  A sphere's *candidate* root -- root1 if root1 > t_min,
// else root2 if root2 > t_min (common.rs:84-92) -- does not depend on t_max,
// and the reference keeps the smallest candidate, first index winning ties.
// So any visiting order that (1) applies the same candidate arithmetic and
// (2) keeps the argmin with an (t, index) tie-break returns the identical
// sphere and t.  Pruning is exact because the point o + t*d of any computed
// candidate lies within  r + K*(|o - c| + r)  of the centre (rounding-error
// bound), so a box inflated by that margin per ray can never
// hide a sphere the brute-force loop would accept.
#pragma once

#include <cstdint>
#include <vector>

#include "scene.h"

namespace rtamd {

// Nodes: two float4 each.  lo = (min.x, min.y, min.z, bits(a)), hi = (max.x,
// max.y, max.z, bits(b)).  Internal: a = left child index (right = a + 1),
// b = split axis.  Leaf: a = first primitive | kLeafBit, b = primitive count.
constexpr uint32_t kLeafBit = 0x80000000u;
constexpr uint32_t kNodeEnd = 0xFFFFFFFFu;

struct SphereBVH {
    std::vector<float> nodes;       // 8 floats per node
    std::vector<uint32_t> miss;     // 8 per node: DFS successor per ray octant
    std::vector<float> prims;       // 4 floats per BVH sphere: (cx, cy, cz, r*r)
    std::vector<uint32_t> prim_id;  // original sphere index (tie-break, shading)
    std::vector<uint32_t> big;      // spheres always tested by brute force (ascending)
    // Per-ray inflation inputs (all rounded up): |o - c| <= |o - centre| + radius
    // for every BVH sphere; rmax = largest BVH radius; mag = largest |coordinate|;
    // inv_rmin >= 1 / smallest BVH radius (the quadratic bound).
    float centre[3] = {0, 0, 0};
    float radius = 0, rmax = 0, mag = 0, inv_rmin = 0;
    uint32_t depth = 0;
};

SphereBVH build_sphere_bvh(const std::vector<Sphere> &spheres, uint32_t leaf_size);

// Triangle BVH for Mesh::hit (common.rs:178-223).  The reference's triangle
// t is (n.o + d)/cos (common.rs:141), so an accepted hit point lies on the
// triangle translated by 2(n^.o)n^ -- a "phantom" copy that depends on the
// ray origin o.  Each node therefore also stores the box of its triangles'
// unit normals; the kernel widens the node box per ray by the interval of
// 2(n^.o)n^ over that normal box plus a rounding margin.
// Nodes: four float4 -- (min.xyz, a) (max.xyz, b) (nmin.xyz, 0) (nmax.xyz, 0)
// with a/b as in SphereBVH.
// Kernel image of a triangle tree's boxes: u16 per coordinate on a per-tree
// grid, decoded as fmaf(q, step, base); lower faces round down and upper faces
// up, so a decoded box always contains the float box (checked by decoding).
struct QuantGrid {
    float base[3] = {0, 0, 0}, step[3] = {1, 1, 1};
};

struct TriangleBVH {
    std::vector<float> nodes;       // 16 floats per node
    std::vector<uint32_t> miss;     // 8 per node
    // 16 floats per BVH triangle, in tree order: (n.x, n.y, n.z, n.v0)
    // (v0, bits(original index)) (v1, 0) (v2, 0)
    std::vector<float> tris;
    std::vector<uint32_t> loose;    // brute-forced triangles (non-finite data, slivers)
    float centre[3] = {0, 0, 0};
    float radius = 0, mag = 0;      // vertices within radius of centre; max |coordinate|
    // Boxes hold the phantoms for origin oc; the kernel widens them by
    // 2(n^.d)n^ with d = o - oc (oc = 0: the plain tree).
    float oc[3] = {0, 0, 0};
    uint32_t depth = 0;
    // kernel nodes, 8 u32: box (6 x u16), normal box (6 x u16), a, link with
    // a = child | axis << 29 (internal) or 1 << 31 | first << 3 | count (leaf)
    // and link = miss[8 * node] (fixed child-a-first order)
    std::vector<uint32_t> qnodes;
    QuantGrid qbox;
    float nbase = -1, nstep = 1;    // normal grid (all three axes)
    // 4-wide image of the same tree (render.hip tri_wide): one 128-B record per
    // wide node, 32 u32: child c's box words (qnodes words 0-2 of the binary
    // node it is) at 6c..6c+2, its normal box at 6c+3..6c+5 as six halves
    // (lo.xyz, hi.xyz, rounded outward from the float normal box), child words
    // at 24..27 -- internal:
    // the child's wide index; leaf: the qnode leaf word (kLeafBit | first << 3 |
    // count); empty slot: kLeafBit (no triangles) -- and 28..31 zero.  Wide
    // node = a binary node's grandchildren (a leaf child stays itself); the
    // root record holds binary node 0's.  Breadth-first, root 0.  Empty when
    // there are more than 65535 wide nodes (the walk's stack holds u16).
    std::vector<uint32_t> wnodes;
    uint32_t wdepth = 0;            // deepest wide node fetched (root 0): stack <= 3 * wdepth
};
// Fills tb.wnodes / tb.wdepth from tb.qnodes (build_triangle_bvh calls it).
void build_wide_image(TriangleBVH &tb);

// Per-origin-cell triangle trees: a grid of cubic cells of
// edge `size` from `lo` (n[0] x n[1] x n[2], cell c = (z n1 + y) n0 + x) over
// the box of the mesh and of the spheres no larger than the mesh.  Tree c
// holds the phantoms of origin = cell c's centre (build_triangle_bvh with oc),
// so a secondary ray whose origin lies in the cell is widened by at most the
// cell's half-diagonal; tree ncells is the static tree (origins outside the
// grid).  Every tree is exact for any origin (the per-ray widening covers
// o - oc), so the choice of tree only changes the work.  All trees share one
// quantisation grid (the union of their root boxes; the static tree tb is
// re-quantised on it), so the kernel's grid parameters stay per launch.  Wide
// images are concatenated with a fixed stride; the records are one array for
// all trees (the static tree's, then copies for cell-tree leaves that are not
// one run of it).
struct TriangleCells {
    float lo[3] = {0, 0, 0};
    float size = 0;
    uint32_t n[3] = {0, 0, 0};
    uint32_t ncells = 0;
    std::vector<uint32_t> wnodes;   // (ncells + 1) x stride_w wide nodes of 32 u32
    std::vector<float> tris;        // records of 16 floats (static tree's first)
    uint32_t stride_w = 0, wdepth = 0;
    float mag = 0;                  // largest |coordinate| over the trees (rho)
};
// Empty (ncells == 0) when a tree has no wide image or the trees do not fit
// the kernel's 32-bit indices.  `size` is the starting edge: it grows until the
// grid has <= 1024 cells and the trees hold <= 4e7 triangles in all.
TriangleCells build_triangle_cells(const std::vector<Triangle> &tris, const std::vector<float> &tri_hot,
                                   const std::vector<Sphere> &spheres, uint32_t leaf_size, float size,
                                   TriangleBVH &tb);
// The smallest cell edge (of a geometric ladder) that cuts the box of the
// mesh's finite vertices into at most max_cells cells; 0 for an empty mesh.
float triangle_cell_edge(const std::vector<Triangle> &tris, uint32_t max_cells);

// tri_hot: PackedScene::tri_hot (the exact per-triangle n and n.v0 bits).
// oc (optional): origin the boxes are built for; phantom: SAH weight of the
// normal spread (<= 0: derived from the scene); image = false: no quantised
// nodes and wide image (build_triangle_cells makes them on its common grid).
TriangleBVH build_triangle_bvh(const std::vector<Triangle> &tris, const std::vector<float> &tri_hot,
                               uint32_t leaf_size, const float *oc = nullptr,
                               double phantom = 0, bool image = true);

// Primary rays all start at the camera origin, so their phantom triangles are
// fixed: this tree holds, per triangle of `tb`, its box translated by
// 2(n^.o)n^ for o = origin and padded by the kernel's margin rho(o), under a
// plain SAH build.  Bounce-0 rays traverse it with an ordinary slab test.
// Nodes as SphereBVH (8 floats); tris/miss as TriangleBVH.  Rebuilt whenever
// the camera moves (load_world, move_camera_position).
struct CameraTriangleBVH {
    std::vector<float> nodes;
    std::vector<uint32_t> miss;
    std::vector<float> tris;
    float origin[3] = {0, 0, 0};
    uint32_t depth = 0;
    std::vector<uint32_t> qnodes;   // kernel nodes, 8 u32: box (6 x u16), a, link, 0 0 0
    QuantGrid qbox;
    std::vector<float> rec_box;     // per record (tris order): padded phantom box lo.xyz, hi.xyz
};
// tree = false: the records and rec_box only (triangle order, no nodes), all
// the primary strip lists need; bounce-0 rays then never walk this tree.
CameraTriangleBVH build_camera_triangle_bvh(const std::vector<Triangle> &tris,
                                            const std::vector<float> &tri_hot, const TriangleBVH &tb,
                                            const float origin[3], uint32_t leaf_size, bool tree = true);

// Primary-ray triangle lists.  A bounce-0 ray of pixel (col, row) starts at
// the camera origin o and points into the pixel's footprint, u in
// [col, col + 1] / (W - 1), v in [row, row + 1] / (H - 1) (common.rs:335-336,
// camera.rs:84-89).  A camera-tree record can only be accepted by such a ray
// if its padded phantom box (rec_box) meets that footprint's frustum, so
// each strip of kTriStripW pixels of one row lists the records whose box
// projects (through o, onto the image plane) near it, with a one-pixel
// margin for the rounding of u, v and the direction.  Boxes not entirely in
// front of the camera go to the `always` list; boxes entirely behind it are
// dropped (a primary ray only reaches points with positive depth).
constexpr uint32_t kTriStripW = 8;
struct PrimaryTriLists {
    std::vector<uint32_t> offsets;  // strips + 1 (CSR over items); the `always`
    std::vector<uint32_t> items;    // records follow at [offsets.back(), items.size())
    uint32_t strips_per_row = 0;
};
PrimaryTriLists build_primary_tri_lists(const CameraTriangleBVH &ct, const CameraModel &cam,
                                        size_t width, size_t height);

// Primary-ray sphere candidates (bounce 0, instead of the sphere-tree walk).
// A primary ray of pixel (col, row) points into that pixel's footprint, so
// only tree spheres whose inflated ball (radius r + K(|o - c| + r) + e_abs, the
// walk's pruning margin) projects onto the footprint can produce
// a candidate.  Each pixel keeps up to kSphListMax such spheres (tree-order
// prim indices); a pixel with more, and every pixel when some ball is not
// entirely in front of the camera, walks the tree instead.  Balls entirely
// behind the camera are dropped.  Candidates keep the (t, index) argmin, so
// the order of the list does not matter (bvh.h header).
constexpr uint32_t kSphListMax = 3;
constexpr uint32_t kSphListWalk = 0xFFFFu;
struct PrimarySphereLists {
    // 2 u32 per image pixel (row 0 = top): (i0 | i1 << 16, i2 | count << 16),
    // count in [0, kSphListMax] or kSphListWalk; empty = lists not usable
    std::vector<uint32_t> rec;
};
PrimarySphereLists build_primary_sphere_lists(const SphereBVH &bv, const CameraModel &cam,
                                              size_t width, size_t height);
// The same build on the device (render.hip launch_sphere_lists): the host
// checks and the per-frame constants; false = no lists (every primary ray walks).
struct SphereListParams {
    double Mi[9];          // inverse camera map, row-major
    double o[3];           // camera origin
    double e_abs, wden, hden;
    uint32_t n, width, height;
};
bool sphere_list_params(const SphereBVH &bv, const CameraModel &cam, size_t width, size_t height,
                        SphereListParams &out);

}  // namespace rtamd
