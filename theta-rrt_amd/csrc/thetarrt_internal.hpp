// Internal declarations shared by kernels.hip and capi.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "../../include/thetarrt.h"
#include "geom.hpp"

#define TR_ST_PENDING 6   /* expansion computed, arc check outstanding (internal) */

namespace tr {

struct NNPart {
  double s;      // squared distance of the chunk's best node (INFINITY if none)
  int64_t idx;   // its index (-1 if none)
};

void launch_samples(hipStream_t st, const Params& P, const Grid& g, const double* gauss, int64_t B,
                    double gx, double gy, double gth, tr_sample* samples, int2* qxy, int32_t* live);
// Node chunks of a sweep: enough blocks to fill the chip, chunks of >= min_chunk nodes (x4).
int64_t nn_chunks(int64_t B, int64_t N, int64_t* chunk, int64_t min_chunk = 256);
void launch_nn_partial(hipStream_t st, const int2* qxy, int64_t B, const double2* txy, int64_t n0,
                       int64_t n1, int64_t chunk, int64_t C, NNPart* part);
void launch_nn_merge(hipStream_t st, const NNPart* part, int64_t C, int64_t B, int64_t* out);
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

}  // namespace tr
