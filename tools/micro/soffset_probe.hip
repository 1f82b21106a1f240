// Probe: does the raw-buffer range check include soffset (gfx950)? and LDS-DMA likewise.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void probe(const int *base, int *out) {
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void *)base, (short)0, 64, 0x00020000);
  int l = threadIdx.x;
  // voffset = 4*l (0..252), soffset = 0 / 32 / 64 / 128
  out[l] = __builtin_amdgcn_raw_buffer_load_b32(r, 4 * l, 0, 0);
  out[64 + l] = __builtin_amdgcn_raw_buffer_load_b32(r, 4 * l, 32, 0);
  out[128 + l] = __builtin_amdgcn_raw_buffer_load_b32(r, 4 * l, 64, 0);
  out[192 + l] = __builtin_amdgcn_raw_buffer_load_b32(r, 0, 4 * l, 0);
}
int main() {
  int h[1024]; for (int i = 0; i < 1024; ++i) h[i] = 1000 + i;
  int *d, *o; hipMalloc(&d, 4096); hipMalloc(&o, 4096);
  hipMemcpy(d, h, 4096, hipMemcpyHostToDevice);
  probe<<<1, 64>>>(d, o);
  int r[256]; hipMemcpy(r, o, 1024, hipMemcpyDeviceToHost);
  const char *nm[4] = {"soff=0", "soff=32", "soff=64", "voff=0,soff=4l"};
  for (int k = 0; k < 4; ++k) { printf("%s:", nm[k]); for (int i = 0; i < 40; i += 2) printf(" %d", r[64 * k + i]); printf("\n"); }
  return 0;
}
