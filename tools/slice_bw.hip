// slice_bw.hip — HBM read bandwidth of the parameter-gradient operand pattern (timing tool).
//
// A wide layer's parameter gradients read, per row, three 800-byte slices: z_l and z_{l+1} from
// the [rows][620] float saves and G_{l+1} from the [rows][640] gradients (2 480 / 2 560-byte
// rows).  This measures how fast a plain streaming kernel reads exactly those slices (dwordx4
// loads, every byte once, a checksum so nothing is elided) against the same byte count read
// contiguously — whether the row-slice pattern itself caps the bandwidth.
//   hipcc --offload-arch=gfx950 -O3 -o tools/slice_bw tools/slice_bw.hip && ./tools/slice_bw
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                               \
    }                                                                         \
  } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));

// slices: rows x (3 slices x 50 float4); item i -> row i / 150, slice (i % 150) / 50, q = i % 50
__global__ void k_slices(const f4* __restrict__ z, const f4* __restrict__ g, int64_t rows, int ldz4, int ldg4,
                         int za4, int zb4, int gb4, float* out) {
  const int64_t n = rows * 150;
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / 150;
    const int k = (int)(i % 150), s = k / 50, q = k % 50;
    const f4 v = s == 0 ? z[r * ldz4 + za4 + q] : s == 1 ? z[r * ldz4 + zb4 + q] : g[r * ldg4 + gb4 + q];
    acc += v;
  }
  const float t = acc[0] + acc[1] + acc[2] + acc[3];
  if (t == 12345.f) out[threadIdx.x] = t;  // never true for the zero-filled inputs; keeps the loads
}

__global__ void k_contig(const f4* __restrict__ a, int64_t n4, float* out) {
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x)
    acc += a[i];
  const float t = acc[0] + acc[1] + acc[2] + acc[3];
  if (t == 12345.f) out[threadIdx.x] = t;
}

int main() {
  const int64_t rows = 204800;
  const int ldz = 620, ldg = 640;
  f4 *z, *g, *c;
  float* out;
  CK(hipMalloc(&z, rows * ldz * 4));
  CK(hipMalloc(&g, rows * ldg * 4));
  const int64_t bytes = rows * 3 * 800;
  CK(hipMalloc(&c, bytes));
  CK(hipMalloc(&out, 4096));
  CK(hipMemset(z, 0, rows * ldz * 4));
  CK(hipMemset(g, 0, rows * ldg * 4));
  CK(hipMemset(c, 0, bytes));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int grids[3] = {1024, 2048, 8192};
  for (int gi = 0; gi < 3; ++gi) {
    const int grid = grids[gi];
    for (int kind = 0; kind < 2; ++kind) {
      for (int w = 0; w < 3; ++w) {
        if (kind == 0)
          k_slices<<<grid, 256>>>(z, g, rows, ldz / 4, ldg / 4, 0, 50, 55, out);
        else
          k_contig<<<grid, 256>>>(c, bytes / 16, out);
      }
      CK(hipEventRecord(e0));
      const int reps = 20;
      for (int rep = 0; rep < reps; ++rep) {
        if (kind == 0)
          k_slices<<<grid, 256>>>(z, g, rows, ldz / 4, ldg / 4, 0, 50, 55, out);
        else
          k_contig<<<grid, 256>>>(c, bytes / 16, out);
      }
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms = 0.f;
      CK(hipEventElapsedTime(&ms, e0, e1));
      ms /= reps;
      printf("{\"kind\": \"%s\", \"grid\": %d, \"MB\": %.1f, \"us\": %.1f, \"GBps\": %.0f}\n",
             kind == 0 ? "row_slices_3x800B" : "contiguous", grid, bytes / 1e6, ms * 1e3, bytes / (ms * 1e-3) / 1e9);
    }
  }
  CK(hipGetLastError());
  return 0;
}
