// Diagnostic microbenchmark (not the product): the store roofline of k_evals' row pattern —
// 262 144 rows of 24 doubles (192 B) written by 16-B stores, 12 lanes per row and 5 rows per
// wave instruction (the row phase's lane map), 512 workgroups x 8 waves, each workgroup one
// contiguous block of rows; R passes over the same buffer in ONE launch (as k_evals' runs), or
// R launches.  Prints us per pass.  hipcc --offload-arch=gfx950 -O3 store_roof.hip -o store_roof
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <vector>
typedef unsigned int v4u __attribute__((ext_vector_type(4)));

template <int AUX>
__global__ __launch_bounds__(512) void k_rows(double* w, int rows, int nblk, int passes, int pass_stride_rows) {
  const int b = blockIdx.x, lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int per = (rows + nblk - 1) / nblk, r0 = b * per, r1 = min(rows, r0 + per);
  const int Lr = 12, R = 5, rr = lane / Lr, col = lane - rr * Lr;
  for (int p = 0; p < passes; ++p) {
    double* wp = w + (size_t)p * pass_stride_rows * 24;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(wp, (short)0, rows * 192, 0x00020000);
    for (int r = r0 + wv * R; r < r1; r += 8 * R) {
      const int row = r + rr;
      const int off = (rr < R && row < r1) ? (row * 24 + 2 * col) * 8 : 0x7fff0000;
      const double x = (double)row, y = (double)p;
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, make_double2(x, y)), rs, off, 0, AUX);
    }
  }
}

int main() {
  const int rows = 262144, nblk = 512, R = 20;
  double* w;
  hipMalloc(&w, (size_t)rows * 192 * R);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int fresh = 0; fresh < 2; ++fresh) {
    for (int rep = 0; rep < 3; ++rep) {
      hipEventRecord(e0);
      hipLaunchKernelGGL(k_rows<16>, dim3(nblk), dim3(512), 0, 0, w, rows, nblk, R, fresh ? rows : 0);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      printf("one launch, %d passes, %s buffer: %.2f us per pass (%.2f TB/s)\n", R, fresh ? "fresh" : "same",
             ms * 1e3 / R, rows * 192.0 * R / (ms * 1e-3) / 1e12);
    }
  }
  for (int rep = 0; rep < 3; ++rep) {
    hipEventRecord(e0);
    for (int p = 0; p < R; ++p) hipLaunchKernelGGL(k_rows<16>, dim3(nblk), dim3(512), 0, 0, w, rows, nblk, 1, 0);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    printf("%d launches of one pass: %.2f us per pass\n", R, ms * 1e3 / R);
  }
  return 0;
}
