// LDS-DMA addressing probe: one wave copies 1 KB from global into LDS at a
// given byte offset with buffer_load_dwordx4 ... lds and with
// global_load_lds_dwordx4, then reads it back.  Prints mismatches per offset.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
__global__ void probe(const float* src, float* out, int off, int mode) {
  __shared__ __attribute__((aligned(16))) char smem[150 * 1024];
  for (int i = threadIdx.x; i < 150 * 256; i += 64) reinterpret_cast<float*>(smem)[i] = -1.0f;
  __syncthreads();
  if (mode == 0) {
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)src, 0, 1024, 0x00020000);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)(smem + off), 16,
                                             threadIdx.x * 16, 0, 0, 0);
  } else {
    __builtin_amdgcn_global_load_lds((const void*)(src + threadIdx.x * 4),
                                     (__attribute__((address_space(3))) void*)(smem + off), 16, 0, 0);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int i = 0; i < 4; ++i) out[threadIdx.x * 4 + i] = reinterpret_cast<float*>(smem + off)[threadIdx.x * 4 + i];
}
int main() {
  std::vector<float> h(256);
  for (int i = 0; i < 256; ++i) h[i] = (float)i;
  float *d, *o;
  hipMalloc(&d, 1024); hipMalloc(&o, 1024);
  hipMemcpy(d, h.data(), 1024, hipMemcpyHostToDevice);
  for (int mode = 0; mode < 2; ++mode)
    for (int off : {0, 1024, 49152, 65536, 70656, 98304, 131072, 146432}) {
      hipMemset(o, 0, 1024);
      hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, o, off, mode);
      std::vector<float> r(256);
      hipMemcpy(r.data(), o, 1024, hipMemcpyDeviceToHost);
      int bad = 0;
      for (int i = 0; i < 256; ++i) bad += r[i] != h[i];
      printf("mode %s off %6d bad %d first %g\n", mode ? "global_lds" : "buffer_lds", off, bad, r[0]);
    }
  return 0;
}
