// Internal declarations shared by kernels.hip, nn.hip, dedupe.hip and capi.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

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
void launch_samples(hipStream_t st, const Params& P, const Grid& g, const double* gauss, int64_t B,
                    double gx, double gy, double gth, tr_sample* samples, int2* qxy, int32_t* live);
void launch_expand(hipStream_t st, const Params& P, const Grid& g, const int64_t* nnidx, int64_t B,
                   const tr_sample* samples, const int32_t* live, const double2* txy,
                   const double* tth, tr_record* rec);
void launch_arc(hipStream_t st, const Params& P, const Grid& g, int64_t B, const double2* txy,
                double gx, double gy, double gth, tr_record* rec);
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
// n_ub = host upper bound on *count (sizes the grid); m32 needs nn_scratch(B, n_ub) floats.
int64_t nn_chunks(int64_t B, int64_t N, int64_t* chunk);
int64_t nn_scratch(int64_t B, int64_t n_ub);
void nn_launch(hipStream_t st, const int2* qxy, int64_t B, const double2* txy, const float2* t32,
               const int64_t* count, int64_t n_ub, const unsigned long long* maxabs, double qmax,
               float* m32, int64_t* out);

// ---- dedupe.hip: device pose table + per-batch scratch
struct DDState {
  int32_t* htab;             // pose -> node index, open addressing, -1 empty
  uint64_t hmask;
  unsigned long long* btab;  // per-batch pose -> (epoch << 32 | first record index)
  uint64_t bmask;
  unsigned long long epoch;  // batch counter (>= 1)
  int32_t *e, *fl, *first, *isfirst, *rank;
  int64_t* count;            // device node count
  int64_t* base;             // node count before the batch (scratch)
  unsigned long long* maxabs;  // bits of max |coordinate| (non-negative double)
};
// out: n commit records in device-accessible (pinned host) memory.
void dd_batch(hipStream_t st, const DDState& d, const tr_sample* smp, const tr_record* rec, int64_t n,
              double2* txy, float2* t32, double* tth, tr_commit_rec* out);
void dd_rebuild(hipStream_t st, const DDState& d, const double2* txy, const double* tth, int64_t N);

}  // namespace tr
