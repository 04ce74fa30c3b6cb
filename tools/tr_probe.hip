// Probe of ds_read_b64_tr_b16 semantics on gfx950: LDS holds a 16 x 64 image of 16-bit values
// v = row * 256 + col; every lane supplies the address the guide's rule gives (lane 4q+p of each
// 16-lane group: row q, columns 4p..4p+3 of the group's 16-column block); prints what each lane
// receives.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef short s16x4 __attribute__((ext_vector_type(4)));
__global__ void probe(short* out, int mode) {
  __shared__ short img[16 * 64];
  for (int i = threadIdx.x; i < 16 * 64; i += 64) img[i] = (short)((i / 64) * 256 + (i % 64));
  __syncthreads();
  const int lane = threadIdx.x, grp = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int row = q + (mode ? 4 * grp : 0), col = 16 * grp + 4 * p;
  s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(img + row * 64 + col));
  for (int j = 0; j < 4; ++j) out[lane * 4 + j] = v[j];
}
int main() {
  short* d;
  short h[256];
  hipMalloc(&d, 512);
  for (int mode = 0; mode < 2; ++mode) {
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, mode);
    hipMemcpy(h, d, 512, hipMemcpyDeviceToHost);
    printf("mode %d (lane: received (row,col) x4)\n", mode);
    for (int l = 0; l < 64; ++l) {
      printf("%2d:", l);
      for (int j = 0; j < 4; ++j) printf(" (%d,%d)", h[l * 4 + j] / 256, h[l * 4 + j] % 256);
      printf(l % 2 ? "\n" : "   ");
    }
  }
  return 0;
}
