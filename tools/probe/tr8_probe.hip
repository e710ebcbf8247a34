// One-off probe (tools/): ds_read_b64_tr_b8 lane/byte mapping and the v_mfma_i32_32x32x32_i8
// operand/result maps, checked against a host model with exact integer data.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
typedef int v2i __attribute__((ext_vector_type(2)));
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
__global__ void k(int hi, int* out) {
  __shared__ unsigned char L[1024];
  for (int i = threadIdx.x; i < 1024; i += 64) L[i] = (unsigned char)(hi ? (i >> 8) : i);
  __syncthreads();
  v2i r = __builtin_amdgcn_ds_read_tr8_b64_v2i32((__attribute__((address_space(3))) v2i*)(L + 8 * threadIdx.x));
  out[2*threadIdx.x] = r.x; out[2*threadIdx.x+1] = r.y;
}
__global__ void m(const v4i* a, const v4i* b, v16i* c) {
  c[threadIdx.x] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[threadIdx.x], b[threadIdx.x], (v16i){}, 0, 0, 0);
}
int main() {
  int *d; hipMalloc(&d, 512 * 4);
  int lo[128], hi[128];
  k<<<1, 64>>>(0, d); hipMemcpy(lo, d, 512, hipMemcpyDeviceToHost);
  k<<<1, 64>>>(1, d); hipMemcpy(hi, d, 512, hipMemcpyDeviceToHost);
  printf("tr8: lane: source byte index of output bytes 0..7\n");
  for (int l = 0; l < 64; l++) {
    printf("%2d:", l);
    for (int j = 0; j < 8; j++) {
      int w = j >> 2, s = 8 * (j & 3);
      int v = ((lo[2*l+w] >> s) & 255) | (((hi[2*l+w] >> s) & 255) << 8);
      printf(" %4d", v);
    }
    printf("\n");
  }
  // MFMA: A[32][32], B[32][32] int8; assume lane l: row/col l&31, k = 16(l>>5) + j
  int8_t A[32][32], B[32][32];
  srand(1);
  for (int i = 0; i < 32; i++) for (int kk = 0; kk < 32; kk++) { A[i][kk] = (int8_t)(rand() % 255 - 127); B[kk][i] = (int8_t)(rand() % 255 - 127); }
  int8_t ha[64][16], hb[64][16];
  for (int l = 0; l < 64; l++) for (int j = 0; j < 16; j++) { ha[l][j] = A[l & 31][16 * (l >> 5) + j]; hb[l][j] = B[16 * (l >> 5) + j][l & 31]; }
  void *da, *db, *dc; hipMalloc(&da, 1024); hipMalloc(&db, 1024); hipMalloc(&dc, 64 * 64);
  hipMemcpy(da, ha, 1024, hipMemcpyHostToDevice); hipMemcpy(db, hb, 1024, hipMemcpyHostToDevice);
  m<<<1, 64>>>((const v4i*)da, (const v4i*)db, (v16i*)dc);
  int hc[64][16]; hipMemcpy(hc, dc, 4096, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int l = 0; l < 64; l++) for (int r = 0; r < 16; r++) {
    int row = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5), col = l & 31;
    long ref = 0; for (int kk = 0; kk < 32; kk++) ref += A[row][kk] * B[kk][col];
    if (ref != hc[l][r]) bad++;
  }
  printf("mfma i8 32x32x32 with k = 16h + j, f32 C map: %d mismatches of 1024\n", bad);
  return 0;
}
