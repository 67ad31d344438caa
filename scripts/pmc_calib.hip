// pmc_calib.hip — calibrates rocprofv3 FETCH_SIZE / WRITE_SIZE on gfx950 for
// the access widths the engine's kernels use (MI355X_MICROARCH.md: only
// 16-B-per-lane streaming reads are calibrated there, at exactly 1/2).
// Each kernel streams exactly 1 GiB of a 4 GiB buffer (past the 256 MiB
// Infinity Cache), coalesced, one element per lane per iteration.
// Build: hipcc -O3 --offload-arch=gfx950 scripts/pmc_calib.hip -o scripts/build/pmc_calib
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s\n", hipGetErrorString(e_)); return 1; } } while (0)

template <class T>
__global__ void k_read(const T* __restrict__ p, size_t n, unsigned long long* out) {
  unsigned long long acc = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const T x = p[i];
    const uint8_t* b = (const uint8_t*)&x;
    acc += b[0] + b[sizeof(T) - 1];
  }
  if (acc == 0xFFFFFFFFFFFFull) out[0] = acc;  // keeps the loads
}
template <class T>
__global__ void k_write(T* __restrict__ p, size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    T x;
    uint8_t* b = (uint8_t*)&x;
    for (size_t k = 0; k < sizeof(T); ++k) b[k] = (uint8_t)(i + k);
    p[i] = x;
  }
}
// read-modify-write of u32 (phase A pass 3's pending counts)
__global__ void k_rmw4(uint32_t* __restrict__ p, size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    p[i] = p[i] + 1u;
}

// phase A's list walk pattern: 400-byte lists (100 four-byte entries) at an
// 8576-byte row stride (FC = 2144 entries), read as 16-byte blocks, one list
// per half-wave here; each list is read once
__global__ void k_lists(const uint8_t* __restrict__ p, int nlist, unsigned long long* out, unsigned long long magic) {
  const int l = blockIdx.x * 2 + (threadIdx.x >> 5);
  const int b = threadIdx.x & 31;
  unsigned long long acc = 0;
  if (l < nlist && b < 25) {
    const uint4 x = *(const uint4*)(p + (size_t)l * 8576 + 16 * b);
    acc = x.x + x.w;
  }
  if (acc == magic) out[0] = acc;  // a runtime value: the loads cannot be proven dead
}

int main() {
  const size_t GiB = 1ull << 30;
  uint8_t* buf = nullptr;
  unsigned long long* out = nullptr;
  CHECK(hipMalloc(&buf, 4 * GiB));
  CHECK(hipMalloc(&out, 8));
  CHECK(hipMemset(buf, 1, 4 * GiB));
  const int grid = 256 * 8 * 4, blk = 256;
  // different GiB-sized regions per kernel, so no kernel re-reads a predecessor's lines
  k_read<uint8_t><<<grid, blk>>>(buf, GiB, out);
  k_read<uint32_t><<<grid, blk>>>((const uint32_t*)(buf + GiB), GiB / 4, out);
  k_read<uint64_t><<<grid, blk>>>((const uint64_t*)(buf + 2 * GiB), GiB / 8, out);
  k_read<uint4><<<grid, blk>>>((const uint4*)(buf + 3 * GiB), GiB / 16, out);
  k_write<uint32_t><<<grid, blk>>>((uint32_t*)buf, GiB / 4);
  k_write<uint64_t><<<grid, blk>>>((uint64_t*)(buf + GiB), GiB / 8);
  k_write<uint4><<<grid, blk>>>((uint4*)(buf + 2 * GiB), GiB / 16);
  k_rmw4<<<grid, blk>>>((uint32_t*)(buf + 3 * GiB), GiB / 4);
  const int nlist = 400000;  // 400000 * 8576 B = 3.4 GB of rows, 160 MB of lists
  k_lists<<<nlist / 2, 64>>>(buf, nlist, out, 0x123456789ull);
  CHECK(hipDeviceSynchronize());
  printf("each kernel streams %zu bytes (rmw4: read and write); k_lists reads %d lists of 400 B "
         "(%d bytes, %d bytes of 128-B lines)\n", GiB, nlist, nlist * 400, nlist * 512);
  CHECK(hipFree(buf));
  CHECK(hipFree(out));
  return 0;
}
