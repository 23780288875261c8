// fetch_calib.hip — calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 for the access
// widths the engine uses (MI355X_MICROARCH.md §HBM: "FETCH_SIZE reports 1/2 of the bytes of a
// 16-B-per-lane streaming read; other widths uncalibrated").  Each kernel moves a known byte
// count through a 1 GiB buffer (4x the Infinity Cache):
//   rd4 / rd8 / rd16   : grid-stride coalesced reads of 4 / 8 / 16 B per lane
//   seg8               : 512-B wave segments (8 B per lane) at pseudo-random segment positions
//                        (engine 6's [edge][lane] message accesses)
//   wr8 / wr16         : coalesced stores of 8 / 16 B per lane;  wseg8 : scattered 512-B segments
// Usage (on the GPU box): rocprofv3 --pmc FETCH_SIZE -- ./fetch_calib ; --pmc WRITE_SIZE likewise.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

template <typename V>
__global__ void rd(const V* __restrict__ p, size_t n, double* out) {
  double acc = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const V v = p[i];
    acc += reinterpret_cast<const double*>(&v)[0] * (sizeof(V) >= 8 ? 1.0 : 0.0) + (sizeof(V) < 8 ? (double)reinterpret_cast<const float*>(&v)[0] : 0.0);
  }
  if (acc == 12345.678) out[0] = acc;  // keeps the loads
}
template <typename V>
__global__ void wr(V* __restrict__ p, size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    V v;
    reinterpret_cast<uint32_t*>(&v)[0] = (uint32_t)i;
    for (int k = 1; k < (int)(sizeof(V) / 4); ++k) reinterpret_cast<uint32_t*>(&v)[k] = 0;
    p[i] = v;
  }
}
// one wave per 512-B segment, segments visited in a pseudo-random order (odd multiplier mod 2^k)
__global__ void seg8(const double* __restrict__ p, size_t nseg, double* out) {
  const int lane = threadIdx.x & 63;
  const size_t wave = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6, nw = ((size_t)gridDim.x * blockDim.x) >> 6;
  double acc = 0;
  for (size_t s = wave; s < nseg; s += nw) {
    const size_t q = (s * 2654435761ull) & (nseg - 1);
    acc += p[q * 64 + lane];
  }
  if (acc == 12345.678) out[0] = acc;
}
__global__ void wseg8(double* __restrict__ p, size_t nseg) {
  const int lane = threadIdx.x & 63;
  const size_t wave = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6, nw = ((size_t)gridDim.x * blockDim.x) >> 6;
  for (size_t s = wave; s < nseg; s += nw) {
    const size_t q = (s * 2654435761ull) & (nseg - 1);
    p[q * 64 + lane] = (double)s;
  }
}

int main() {
  const size_t bytes = 1ull << 30;
  void* buf;
  double* out;
  CK(hipMalloc(&buf, bytes));
  CK(hipMalloc(&out, 64));
  CK(hipMemset(buf, 0, bytes));
  CK(hipDeviceSynchronize());
  const dim3 g(256 * 16), b(256);
  hipLaunchKernelGGL(rd<float>, g, b, 0, 0, (const float*)buf, bytes / 4, out);
  hipLaunchKernelGGL(rd<double>, g, b, 0, 0, (const double*)buf, bytes / 8, out);
  hipLaunchKernelGGL(rd<double2>, g, b, 0, 0, (const double2*)buf, bytes / 16, out);
  hipLaunchKernelGGL(seg8, g, b, 0, 0, (const double*)buf, bytes / 512, out);
  hipLaunchKernelGGL(wr<double>, g, b, 0, 0, (double*)buf, bytes / 8);
  hipLaunchKernelGGL(wr<double2>, g, b, 0, 0, (double2*)buf, bytes / 16);
  hipLaunchKernelGGL(wseg8, g, b, 0, 0, (double*)buf, bytes / 512);
  CK(hipDeviceSynchronize());
  printf("each kernel moves %zu bytes (1 GiB)\n", bytes);
  return 0;
}
