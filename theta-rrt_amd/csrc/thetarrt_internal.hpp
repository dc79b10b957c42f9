// Internal declarations shared by kernels.hip, nn.hip, dedupe.hip and capi.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <functional>
#include <string>
#include <vector>

#include "../../include/thetarrt.h"
#include "geom.hpp"

#define TR_ST_PENDING 6   /* expansion computed, arc check outstanding (internal) */

// Per-record resolution flags of the device bookkeeping (dedupe.hip) = the public TR_RS_*.
#define TR_CI_MEMBER TR_RS_MEMBER
#define TR_CI_SAME_NEAR TR_RS_SAME_NEAR
#define TR_CI_FIRST TR_RS_FIRST
typedef tr_resolved tr_commit_rec;   // written by the device into pinned host memory

namespace tr {

// ---- kernels.hip
// zero (optional): a device counter set to 0 by the launch.
void launch_samples(hipStream_t st, const Params& P, const Grid& g, const double* gauss, int64_t B,
                    double gx, double gy, double gth, tr_sample* samples, int2* qxy, int32_t* live,
                    int32_t* zero = nullptr);

void launch_arc_batch(hipStream_t st, const Grid& g, const double* in10, int64_t n, uint8_t* out,
                      int32_t* err);
void launch_los_i32(hipStream_t st, const Grid& g, const int32_t* seg, int64_t n, uint8_t* out,
                    int32_t* err);
void launch_los_f64(hipStream_t st, const Grid& g, const double* seg, int64_t n, uint8_t* out,
                    int32_t* err);
void launch_steer(hipStream_t st, const Params& P, const double* in6, int64_t n, double* out9);
void launch_drive(hipStream_t st, const Params& P, const double* in9, int64_t n, double* out3,
                  int32_t* ok);
void launch_body(hipStream_t st, const Params& P, const Grid& g, const double* xyt, int64_t n,
                 double mult, uint8_t* out, int32_t* err);
void launch_bresenham_list(hipStream_t st, const double* seg, int64_t* out, int64_t cap,
                           int64_t* count);
void launch_circle_list(hipStream_t st, const Grid& g, double cx, double cy, double r,
                        const double* arc10, int64_t* out, int64_t cap, int64_t* count);

// ---- nn.hip: nearest node for B integer queries against the device tree [0, *count)
// NN screen operand of a node: coordinates relative to the tree centre (cx, cy) rounded to fp32,
// and fp32 of their squared norm (nn.hip states the error bound this layout is screened with).
__host__ __device__ inline float4 screen_node(double x, double y, int32_t cx, int32_t cy) {
  const float a = (float)(x - (double)cx), b = (float)(y - (double)cy);
  const double w = (double)a * (double)a + (double)b * (double)b;   // products exact in fp64
  return make_float4(a, b, (float)w, 0.0f);
}
// Threshold on s for sample p = q - centre (exact integers), from the minimum m of s over the tree.
// Eg = 24 u X^2 bounds |s_i - (d_i - |p|^2)| for every node.  The winner w and the node k that
// attains m both have d <= Dup = m + |p|^2 + Eg, i.e. lie within R = sqrt(Dup) of q, so their
// rounding errors obey a bound in terms of |p| and R only (much tighter for samples near the
// centre):  w^ rounding u1 Wp, inner fma u T, outer fma u Sm, fp32 coordinates rep.
__device__ __forceinline__ double screen_E(double px, double py, double R, double Eg) {
  const double u = 5.9604644775390625e-08, u1 = u + 2.220446049250313e-16;   // 2^-24, + 2^-52
  const double p2 = px * px + py * py;
  const double Ax = (fabs(px) + R) * (1.0 + 2.0 * u1), Ay = (fabs(py) + R) * (1.0 + 2.0 * u1);
  const double R1 = R + u1 * fmax(Ax, Ay);                       // |fp32 coordinate - p| bound
  const double Wp = (Ax * Ax + Ay * Ay) * (1.0 + 4.0 * u1);      // >= |w^|
  const double T = fmax(Ax * Ax + R1 * R1, py * py) + u1 * Wp;   // >= |inner fma before rounding|
  const double Sm = p2 + 2.0 * R1 * R1 + u1 * Wp + u * T + 1.0;   // >= |outer fma before rounding|
  const double rep = 2.0 * u1 * (Ax * (2.0 * R1 + u1 * Ax) + Ay * (2.0 * R1 + u1 * Ay));
  return fmin(Eg, 1.25 * (u1 * Wp + u * T + u * Sm + rep));
}

__device__ __forceinline__ double screen_Eg(double X) {
  return 24.0 * 5.9604644775390625e-08 * X * X;                  // 24 u X^2: every node
}

// |centred coordinate| the screen bound needs (tracked as the max over the tree).
__host__ __device__ inline double centred_abs(double x, double y, int32_t cx, int32_t cy) {
  return fmax(fabs(x - (double)cx), fabs(y - (double)cy));
}
// A query = sweep of nodes [0, *hi) writing chunk minima into m32, then the resolve.  The plan
// (chunking) is sized from a host upper bound n_ub of the node count.  qmax bounds |q - centre|.
struct NNPlan {
  int64_t chunk = 0, cmax = 0;
};
NNPlan nn_plan(int64_t B, int64_t n_ub);
int64_t nn_scratch(int64_t B, const NNPlan& p);    // floats of m32
int64_t nn_scratch_ub(int64_t B, int64_t n_ub);    // the most any plan for <= n_ub nodes needs
// nq_p (optional): the sweep and its resolve take only the first *nq_p samples of qxy (a list
// filled on the device), and the resolve writes sample j's result to out[map[j]].
void nn_sweep(hipStream_t st, const int2* qxy, int64_t B, int32_t cx, int32_t cy, const float4* t4,
              const int64_t* hi_p, const NNPlan& p, float* m32, const int32_t* nq_p = nullptr);
// pub (optional): the last block to finish stores pub_v into *pub (release), counting finished
// blocks in *pub_blocks (reset by that block) -- a stream gate on the look-ahead without a
// separate k_publish launch.
struct ResolvePub {
  unsigned long long* flag = nullptr;
  unsigned long long v = 0;
  int32_t* blocks = nullptr;
};
void nn_resolve(hipStream_t st, const int2* qxy, int64_t B, int32_t cx, int32_t cy,
                const double2* txy, const int64_t* count, const NNPlan& p,
                const unsigned long long* maxabs, double qmax, const float* m32, int64_t* out,
                double* dout, ResolvePub pub = ResolvePub(), const int32_t* nq_p = nullptr,
                const int32_t* map = nullptr);
// Exact correction by the nodes [snap, count) appended since a look-ahead resolve (k_nn_delta).
void nn_delta(hipStream_t st, const int2* qxy, int64_t B, const double2* txy, const int64_t* snap_p,
              const int64_t* count, const int32_t* live, int64_t* near, double* dnear,
              int32_t* changed, int32_t* n_changed);
// sweep of [0, count) + resolve (n_ub = host upper bound on *count).
void nn_launch(hipStream_t st, const int2* qxy, int64_t B, int32_t cx, int32_t cy,
               const double2* txy, const float4* t4, const int64_t* count, int64_t n_ub,
               const unsigned long long* maxabs, double qmax, float* m32, int64_t* out,
               double* dout = nullptr);

// ---- dedupe.hip: device pose table + per-batch scratch
struct PoseSlot {           // pose table slot (32 B): key = exact pose bits, idx = node (-1 empty)
  double x, y, th;
  int32_t idx, pad;
};
// Exact-value pose keys (the reference's dict keys, rrt.py:151,179: -0.0 == 0.0).
__device__ __forceinline__ uint64_t pbits(double v) {
  return v == 0.0 ? 0ull : (uint64_t)__double_as_longlong(v);   // -0.0 == 0.0 (Python keys)
}
__device__ __forceinline__ uint64_t fmix(uint64_t h) {
  h ^= h >> 33;
  h *= 0xff51afd7ed558ccdull;
  h ^= h >> 33;
  h *= 0xc4ceb9fe1a85ec53ull;
  return h ^ (h >> 33);
}
__device__ __forceinline__ uint64_t pose_hash(double x, double y, double t) {
  return fmix(pbits(x) ^ fmix(pbits(y) + 0x9E3779B97F4A7C15ull) ^ fmix(pbits(t) + 0x632BE59BD9B4E019ull));
}
__device__ __forceinline__ bool pose_eq(double ax, double ay, double at, double bx, double by,
                                        double bt) {
  return pbits(ax) == pbits(bx) && pbits(ay) == pbits(by) && pbits(at) == pbits(bt);
}

// Pose table: PoseSlot {x, y, th, idx} (idx -1 = empty, the key in the slot), in buckets of
// POSE_BUCKET = 4 slots = one 128-byte line.  A pose's home bucket is hash & (buckets - 1); an
// insert takes the first empty slot of the home bucket, or of the next bucket with one (CAS on idx,
// then the key: lookups and inserts run in different kernels, the tree grows only in the dedupe).
// A lookup reads whole buckets from the home bucket on and stops at the pose or at a bucket with
// an empty slot (nothing is ever removed, so the pose cannot lie beyond one): at a load <= 1/2
// that is one line per lookup almost always, where a linear probe from an arbitrary slot read
// four to five.  Every probe loop is bounded by the table size: a full table (which the host's
// sizing rules out) sets a bit in *err instead of spinning; the commit records carry it to the
// host replay.
constexpr int POSE_BUCKET = 4;
#define TR_DDE_LOOKUP 1  /* TR_DDE_*: a probe loop ran through a whole table */
#define TR_DDE_CLAIM 2
#define TR_DDE_FIRST 4
#define TR_DDE_INSERT 8
#define TR_DDE_GATE 16   /* a stream gate (k_gate) timed out waiting for the other stream */
// Every bounded device-side wait (k_gate, the gate at the end of k_dd, k_dd's waits for earlier
// blocks) gives up after this many ticks of the 100 MHz wall clock: 30 s.
constexpr unsigned long long GATE_TICKS = 3000000000ull;
constexpr int DD_BLOCK = 256;   // records per dedupe block (dedupe.hip; sizes the host's scratch)

// ---- dedupe.hip: one batch's device bookkeeping and the compact delta the host replays
struct DNode {                   // a new node: pose, cameFrom (parent, u) from its last record
  double x, y, th, u[5];
  int32_t parent, straight;
};
struct DEdge { int32_t par, child; };   // G[qnear].append(qnew), in sample order
struct DUpd {                    // cameFrom overwrite of a snapshot node re-reached
  double u[5];
  int32_t idx, parent, straight, pad;
};
struct DHead {                   // counts of the delta; special = replay the resolved records
  int64_t n_new, n_edge, n_upd, special, n, base;
  int32_t err, pad;              // TR_DDE_* bits; pad = head_tag(the dedupe's epoch)
};
// The head names the dedupe that wrote it: the replay worker takes a slot's head only once it
// carries the epoch it waits for (a head of the slot's earlier use is not this batch's).
__host__ __device__ inline int32_t head_tag(unsigned long long epoch) { return (int32_t)(epoch & 0x7fffffffull); }
struct CommitOut {               // one commit slot (pinned, written by the device)
  DHead* head;
  DNode* nodes;
  DEdge* edges;
  DUpd* upd;
  tr_resolved* res;              // special batches only
};
// Batch table of the new poses: slots (epoch << 32 | first record) claimed by CAS + atomicMin,
// blast (epoch << 32 | last record) by atomicMax (three-kernel dedupe only; nullptr: none); another
// epoch's value is an empty slot, so the tables are never cleared (epoch = batch counter, never 0).
struct DDClaim {
  unsigned long long *btab, *blast;
  uint64_t bmask;
  unsigned long long epoch;
  unsigned long long* special;   // atomicMax'ed to epoch by a record the replay must see in order
  int32_t straight_reject;
};
__device__ __forceinline__ bool rec_accepted(const tr_record& r) {
  return r.status == TR_ST_OK && !(r.flags & TR_FL_MEMBER);
}
__device__ __forceinline__ bool rec_new(const tr_record& r) { return rec_accepted(r) && r.ex < 0; }
// a record the sequential replay must see (the reference raises, or stops at the goal, there)
__device__ __forceinline__ bool rec_special(const tr_record& r, int32_t straight_reject) {
  const bool member = (r.flags & TR_FL_MEMBER) != 0;
  if (r.status == TR_ST_INDEX) return (r.flags & TR_FL_INDEX_SAMPLE) || !member;
  if (member) return false;
  if (r.status == TR_ST_STRAIGHT) return !straight_reject;
  return r.status == TR_ST_OK && (r.flags & TR_FL_GOAL);
}
// Claim of record j's new pose (records written by an earlier kernel: relaxed atomics suffice;
// the atomicMin / atomicMax results are unused, so they do not lengthen the chain); returns its
// batch-table slot, -1 for records without a new pose.
__device__ __forceinline__ int32_t dd_claim_one(const DDClaim& c, const tr_record* rec, int64_t j,
                                               const tr_record& r, int32_t* err) {
  const unsigned long long ep = c.epoch, mine = (ep << 32) | (unsigned long long)j;
  if (rec_special(r, c.straight_reject)) atomicMax(c.special, ep);
  if (!rec_new(r)) return -1;
  uint64_t p = pose_hash(r.x, r.y, r.th) & c.bmask;
  for (uint64_t it = 0; it <= 2 * c.bmask + 1; ++it) {
    unsigned long long v = c.btab[p];
    if ((v >> 32) != ep) {
      const unsigned long long old = atomicCAS(&c.btab[p], v, mine);
      if (old == v) {
        if (c.blast) atomicMax(&c.blast[p], mine);
        return (int32_t)p;                     // claimed
      }
      v = old;
      if ((v >> 32) != ep) continue;           // raced to a stale value: retry the slot
    }
    const tr_record& o = rec[(int64_t)(v & 0xffffffffull)];
    if (pose_eq(o.x, o.y, o.th, r.x, r.y, r.th)) {
      atomicMin(&c.btab[p], mine);
      if (c.blast) atomicMax(&c.blast[p], mine);
      return (int32_t)p;
    }
    p = (p + 1) & c.bmask;
  }
  atomicOr(err, TR_DDE_CLAIM);
  return -1;
}
// Cross-block signalling inside a kernel.  MI355X has one L2 per XCD and the L2s are not coherent
// with each other: an agent-scope fence (__threadfence) writes back AND invalidates the whole L2
// of the XCD it runs on (buffer_wbl2 sc1 + buffer_inv sc1), for every kernel running there, so a
// fence per thread stalls the whole chip.  Data one block hands to another in the same kernel
// therefore travels in agent-scope atomic stores / loads (sc1: coherent, nothing else flushed), a
// block signals with one thread after every wave has waited for its own stores and a barrier, and
// a full-L2 write-back (release_l2) happens once per block, only where plain stores must become
// visible to another stream's kernel before this one ends.  An sc1 store is read with sc1 loads
// only: a later kernel's plain load of a line written by sc1 stores returned a stale value
// (measured: the node count in k_dd, tests/test_gpu_bench_parity.py cfg5_w2).  The node counts
// themselves (plain stores of the dedupe's last block, written back before it signals) are read
// with sc1 loads everywhere: a load that cannot be served from a line this XCD cached earlier.
template <class T>
__device__ __forceinline__ void st_sc1(T* p, T v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <class T>
__device__ __forceinline__ T ld_sc1(const T* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void wave_stores_done() { __builtin_amdgcn_s_waitcnt(0); }
__device__ __forceinline__ void release_l2() { __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent"); }
__device__ __forceinline__ void release_sys() { __builtin_amdgcn_fence(__ATOMIC_RELEASE, ""); }

// Spatial index of the nodes each dedupe appends (the look-ahead correction's candidates): square
// bins of 2^shift pixels over the map, DB_CAP inline items per bin, one set of bins per dedupe epoch
// in a ring of four (a look-ahead is at most three dedupes old).  Most bins hold two or three nodes;
// the bins at the map's corners and borders, where clipped samples land, take dozens per batch.  k_dd adds every new node to its
// bin of set epoch & 3 (slot by atomicAdd on the bin's count) and zeroes the counts of set
// (epoch + 1) & 3 for the next dedupe.  Nodes past a bin's DB_CAP items go to the set's overflow
// list (its count is entry nbx * nby of the set's counts): a reader that meets a count above
// DB_CAP also tests that list, and only past the list's capacity scans the appended nodes.  Bin coordinates clamp floor(x), floor(y)
// into the map, which is monotone: a node with |x - qx| <= R lies in a bin column between those
// of qx - R and qx + R whatever its coordinates.
struct DBItem { double x, y; int32_t idx, pad; };
constexpr int DB_CAP = 64;         // items per bin
constexpr int DB_LIGHT = 4;        // a bin of up to this many items is read by one lane in one round
constexpr int DB_LANE = 16;        // bins per lane a sample's box may cover before it scans the nodes
struct DeltaBins {
  uint32_t* cnt = nullptr;         // [4][nbx * nby + 1]
  DBItem* items = nullptr;         // [4][nbx * nby][DB_CAP]
  DBItem* ovf = nullptr;           // [4][ovf_cap]
  int32_t ovf_cap = 0;
  int32_t shift = 0, nbx = 0, nby = 0;
  int32_t xmax = 0, ymax = 0;      // H - 1, W - 1 (x runs over shape[0], search.py:17-24)
};
__device__ __forceinline__ int32_t db_coord(double v, int32_t vmax) {   // clamp(floor(v), 0, vmax)
  const double f = floor(v);
  return f <= 0.0 ? 0 : (f >= (double)vmax ? vmax : (int32_t)f);
}

// ---- nn_grid.hip: the nearest node from a cell grid over the map instead of a sweep of every
// node (same result, bit for bit).  Cells of 2^cs pixels in Morton order over a padded P x P grid;
// cnt / start / shift hold P * P + 1 words (cnt all zero between builds), items one entry per node
// (pad = its cell), rank one word per node.  A build reads the last build's start_old / items_old /
// built_old[0] (nodes grouped so far; nothing of them when `full`) and writes start / items /
// built_new[0]; the host alternates the two.
struct NNGrid {
  uint32_t* cnt = nullptr;
  uint32_t* shift = nullptr;
  uint32_t* rank = nullptr;
  const uint32_t* start_old = nullptr;
  uint32_t* start = nullptr;
  const DBItem* items_old = nullptr;
  DBItem* items = nullptr;
  const int64_t* built_old = nullptr;
  int64_t* built_new = nullptr;
  // optional: samples whose second pass is long go to this list (far_n zeroed by the build,
  // far_j / far_q = sample index and pixel) for a sweep over the list, instead of a block-wide scan
  int32_t* far_n = nullptr;
  int32_t* far_j = nullptr;
  int2* far_q = nullptr;
  uint32_t far_min = 0;                 // nodes of a second pass from which the sample goes to the list
  unsigned long long* part = nullptr;   // the scan's block sums (nn_grid_scan_blocks words), tagged
  uint32_t serial = 0;                  // the build's number (never 0)
  int32_t* err = nullptr;               // TR_DDE_* bits
  int32_t full = 1;
  int32_t cs = 0, P = 0;
  int32_t xmax = 0, ymax = 0;      // H - 1, W - 1
};
void nn_grid_plan(NNGrid& g, int64_t H, int64_t W, int64_t n_ub);   // cs, P, xmax, ymax
// cell lists of the nodes [0, *hi_p) (n_ub: host upper bound of *hi_p, sizes the launch)
void nn_grid_build(hipStream_t st, const NNGrid& g, const double2* txy, const int64_t* hi_p,
                   int64_t n_ub);
// out[j] = nearest node of qxy[j] among the nodes of the build, dout[j] its exact d (optional)
// (live, optional: samples with live[j] != 1 get out[j] = -1 and are not searched)
// (sc1: the results are read by another stream's kernel before this stream's next kernel boundary
// is known to it: coherent stores, as with pub)
void nn_grid_query(hipStream_t st, const NNGrid& g, const int2* qxy, const int32_t* live, int64_t B,
                   int64_t* out, double* dout, ResolvePub pub = ResolvePub(), bool sc1 = false);
int64_t nn_grid_scan_blocks(const NNGrid& g);   // words of NNGrid::part a plan needs

struct DDArgs {
  const tr_record* rec;
  int64_t n;
  double2* txy;
  float4* t4;
  double* tth;
  int64_t* count;                // device node count
  int64_t* snap;                 // slot receiving the node count after this batch
  PoseSlot* htab;                // pose -> node index, open addressing
  uint64_t hmask;
  unsigned long long* maxabs;    // bits of max |centred coordinate| (non-negative double)
  int32_t cx, cy;                // tree centre of the NN screen
  int32_t* err;                  // TR_DDE_* bits, sticky
  DDClaim claim;
  int32_t* slot;                 // per record: batch-table slot of its new pose (-1)
  int32_t* lr;                   // per record: block-local ranks (node, edge, update)
  int32_t* bc;                   // per block: counts (node, edge, update)
  int64_t* base;                 // node count before the batch
  CommitOut out;
  unsigned long long* done;      // the last block of k_dd_emit stores epoch here (stream waits)
  int32_t* blocks;               // k_dd_emit blocks finished (reset by the last one)
  unsigned long long* ready;     // pinned host flag: the last block stores epoch once the commit
                                 // slot is complete and visible to the host (or nullptr)
  // one-kernel dedupe (k_dd): block tickets, per-block status words (epoch-tagged stage + counts),
  // per-record node index (read back by the last block of a special batch)
  int32_t* ticket;
  unsigned long long* bst;
  int64_t* idxs;
  // the next batch's stream gate, taken by k_dd's last block after it has published this batch
  // (the next expansion then needs no k_gate launch): *gate >= gate_v; gate == nullptr: none
  const unsigned long long* gate;
  unsigned long long gate_v;
  DeltaBins bins;                // cnt == nullptr: no index for this epoch
};
// fused = true: one kernel (k_dd: claim, wait for the earlier blocks' claims, count, look back
// over the earlier blocks' counts, emit); false: three kernels (claim / count / emit).
void dd_batch(hipStream_t st, const DDArgs& a, bool fused = true);
// Cross-stream edges without events: k_gate (one thread) holds its stream until *flag >= target
// (sets TR_DDE_GATE in err after GATE_TICKS instead of hanging), k_publish stores v
// into *flag (release) once the stream's earlier kernels are done.
void launch_gate(hipStream_t st, const unsigned long long* flag, unsigned long long target, int32_t* err);
void launch_publish(hipStream_t st, unsigned long long* flag, unsigned long long v);
void launch_handshake(hipStream_t st, unsigned long long* mine, const unsigned long long* other,
                      unsigned long long ticks, unsigned long long* ok);
void dd_rebuild(hipStream_t st, PoseSlot* htab, uint64_t hmask, int32_t* err, const double2* txy,
                const double* tth, int64_t N);

// ---- kernels.hip
// rrt.py:155-176 for B samples (steer, body rays, drive, arc check + goal flag), one record each;
// list / n_list (device, optional): only samples list[0 .. *n_list) (the look-ahead fix-up).
// The snapshot lookups of the dedupe (rrt.py:151,179,187) ride along: TR_FL_MEMBER,
// TR_FL_SAME_NEAR and ex against the pose table htab (NULL: none).
// delta (optional, snap == nullptr: none): a look-ahead's nearest node nnidx[j] with its exact d
// dnear[j] against the snapshot [0, *snap) is first corrected by the nodes [*snap, *count) appended
// since (k_nn_delta's rule: a later node wins only with a strictly smaller sqrt(d)), by each wave
// for its samples, inside the expansion kernel.
struct DeltaArgs {
  const int64_t* snap = nullptr;
  const int64_t* count = nullptr;
  const double* dnear = nullptr;
  // the fp32 screen of the appended nodes (their t4 operands, the coordinate bound of the NN
  // screen): only nodes it cannot rule out get the exact fp64 test
  const float4* t4 = nullptr;
  const unsigned long long* maxabs = nullptr;
  double qmax = 0;
  int32_t cx = 0, cy = 0;
  // the appended nodes by bin (cnt == nullptr: none): every dedupe epoch in [e_lo, e_hi] that
  // appended [*snap, *count) has its set; each sample then tests only the bins its disc covers
  DeltaBins bins;
  unsigned long long e_lo = 0, e_hi = 0;
};
void launch_expand_arc(hipStream_t st, const Params& P, const Grid& g, const int64_t* nnidx,
                       int64_t B, const tr_sample* samples, const int32_t* live, const double2* txy,
                       const double* tth, double gx, double gy, double gth, const PoseSlot* htab,
                       uint64_t hmask, int32_t* err, tr_record* rec, DeltaArgs delta = DeltaArgs());

// ---- findnearest.hip: rrt.py:117-128 for G goals over E edges (parent, child node index); node
// poses read as xs[c * sx], ys[c * sy], ths[c * sth].  scratch: fn_scratch(E, G) bytes.
int64_t fn_blocks(int64_t E, int64_t G);
int64_t fn_scratch(int64_t E, int64_t G);
void launch_findnearest(hipStream_t st, const double* xs, int sx, const double* ys, int sy,
                        const double* ths, int sth, const int64_t* e_par, const int64_t* e_child,
                        int64_t E, const double* goals3, int64_t G, double w, void* scratch,
                        int64_t* out_child, double* out_d);

// ---- astar.hip: search.py:221-307 on the host, lazy Theta*'s line of sight through `los`
// ((x0, y0, x1, y1) -> *clear; returns a TR_* status).
typedef std::function<int(int64_t x0, int64_t y0, int64_t x1, int64_t y1, bool* clear)> LosFn;
struct AStarStats {
  int64_t expanded = 0;      // len(closedSet) when the goal is reached
  int64_t los_segments = 0;  // line-of-sight tests
  int32_t status = 0;        // 0 found, 1 start/goal not valid, 2 inside an obstacle, 3 no path
};
int astar_run(const uint8_t* free_yx, int64_t H, int64_t W, int64_t sx, int64_t sy, int64_t gx,
              int64_t gy, bool theta, const LosFn& los, std::vector<int64_t>& path, AStarStats& st,
              std::string& msg);

// ---- astar_dev.hip: the same search resident on the device, one wave per (start, goal) query.
// work: astar_dev_bytes_per_query(H, W, far_cap) * nq bytes; the caller zeroes the cell words
// (astar_dev_cells) on the stream first.  sg4 / path_xy / path_len / stats are device arrays.
int64_t astar_dev_bytes_per_query(int64_t H, int64_t W, int64_t far_cap);
void astar_dev_cells(int64_t H, int64_t W, int64_t far_cap, int64_t nq, int64_t* off, int64_t* bytes);
void launch_astar_dev(hipStream_t st, const Grid& g, const int32_t* sg4, int64_t nq, int theta,
                      void* work, int64_t far_cap, int64_t* path_xy, int64_t cap,
                      int64_t* path_len, int64_t* stats);

// ---- rng.hip: numpy's legacy gaussian stream on the device (rand_conf's draws, rrt.py:58,66)
struct RngPos {              // stream position: next MT19937 word + numpy's cached gaussian
  int64_t wpos;
  int32_t has, pad;
  double gauss;
};
int64_t rng_attempts_ub(int64_t n);          // worst-case polar attempts for n gaussians
int64_t rng_counts_len(int64_t n);           // int32 scratch of rng_chunk
// n gaussians from *start into out; bstate[b] = position after out[0 .. (b + 1) blen); the ring
// (rs words, a multiple of 624) is topped up past start->wpos + 4 rng_attempts_ub(n) words.
// seeds (15 x 624 words) / done (one zeroed counter): scratch of the parallel generation, which
// chunks of rng_ring_extra(n) > 0 use; the ring then needs that many words more.
void rng_chunk(hipStream_t st, uint32_t* ring, int64_t rs, int64_t* gen_end, const RngPos* start,
               int64_t n, int64_t blen, double* out, RngPos* bstate, int32_t* counts, int32_t* err,
               uint32_t* seeds, int32_t* done);
int64_t rng_ring_extra(int64_t n);
// keys[b * 624 ..] = the key block of bstate[b] (b < nb); rng_rebase re-seeds the stream at *src
// from such a kept block (ring block 0, generation restarts after it).
void rng_keep(hipStream_t st, const uint32_t* ring, int64_t rs, const RngPos* bstate, int64_t nb,
              uint32_t* keys);
void rng_rebase(hipStream_t st, uint32_t* ring, int64_t* gen_end, RngPos* pos0, const RngPos* src,
                const uint32_t* key);

}  // namespace tr
