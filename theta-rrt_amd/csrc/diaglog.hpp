// Diagnosis builds only (build.py --variant phases): a per-translation-unit log of block start /
// end times (100 MHz wall clock), one entry per block, read back through the TU's export function.
// Nothing of this exists in the product build.
#pragma once
#ifdef TR_DIAG_PHASES
#include <hip/hip_runtime.h>
#include <stdint.h>
namespace tr {
constexpr int DLOG_CAP = 1 << 16;
struct DLogEntry { unsigned long long id, t0, t1; };
static __device__ DLogEntry g_dlog[DLOG_CAP];
static __device__ unsigned int g_dlogn;
__device__ __forceinline__ void dlog(unsigned long long id, unsigned long long t0) {
  const unsigned int i = atomicAdd(&g_dlogn, 1u) % DLOG_CAP;
  g_dlog[i] = DLogEntry{id, t0, (unsigned long long)wall_clock64()};
}
}  // namespace tr
#define TR_DLOG_T0 const unsigned long long dlog_t0 = wall_clock64()
#define TR_DLOG(id) do { if (threadIdx.x == 0) tr::dlog(id, dlog_t0); } while (0)
#define TR_DLOG_EXPORT(name)                                                                     \
  extern "C" int name(void* out, unsigned int* n) {                                              \
    if (hipMemcpyFromSymbol(n, HIP_SYMBOL(tr::g_dlogn), sizeof(unsigned int)) != hipSuccess) return 1; \
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(tr::g_dlog), sizeof(tr::g_dlog));            \
  }
#else
#define TR_DLOG_T0
#define TR_DLOG(id)
#define TR_DLOG_EXPORT(name)
#endif
