// probe: LDS layout written by global_load_lds_dwordx3, and raw buffer loads with OOB offsets
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x4 __attribute__((ext_vector_type(4)));
__global__ void k(const float* g, float* o) {
  __shared__ float l[1024];
  for (int i = threadIdx.x; i < 1024; i += 64) l[i] = -1.f;
  __syncthreads();
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(g + threadIdx.x * 3),
                                   (__attribute__((address_space(3))) void*)(l), 12, 0, 0);
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  for (int i = threadIdx.x; i < 256; i += 64) o[i] = l[i];
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)g, (short)0, 1024, 0x00020000);
  f32x4 v = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, threadIdx.x < 8 ? threadIdx.x * 16 : 0x7fffffff, 0, 0));
  o[256 + threadIdx.x * 4 + 0] = v[0]; o[256 + threadIdx.x * 4 + 1] = v[1];
  o[256 + threadIdx.x * 4 + 2] = v[2]; o[256 + threadIdx.x * 4 + 3] = v[3];
}
int main() {
  float h[1024]; for (int i = 0; i < 1024; ++i) h[i] = i;
  float *g, *o; hipMalloc(&g, 4096); hipMalloc(&o, 4096);
  hipMemcpy(g, h, 4096, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, g, o);
  float r[512]; hipMemcpy(r, o, 2048, hipMemcpyDeviceToHost);
  printf("lds[0..40]:"); for (int i = 0; i < 40; ++i) printf(" %g", r[i]); printf("\n");
  printf("lds[180..200]:"); for (int i = 180; i < 200; ++i) printf(" %g", r[i]); printf("\n");
  printf("buf lane0..9:"); for (int i = 0; i < 40; ++i) printf(" %g", r[256 + i]); printf("\n");
  return 0;
}
