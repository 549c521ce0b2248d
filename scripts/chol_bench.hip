// Latency microbenchmark of the register-row SPD factor + solve on one wave (the Newton
// Hessian of a heavy world).  One workgroup per "world"; s_memtime per world.  Measured
// and dropped: a block-parallel factor on a leaves-first dof order
// and a chunked-LTR factor (chunk registers, rank-4 updates).
// build: hipcc -O3 --offload-arch=gfx950 -I mjlab-1_amd/csrc -I scripts -o scripts/chol_bench scripts/chol_bench.hip
// modes: 0 engine (branch-free), 1 pre-round-3 forms, 3 factor only, 4 load_factor + solve
// only, 5 factor only in the latency form (rows_chol<NR, true>), 6 tree form (reversed dof
// order, rows_chol_tree) factor + solve, 7 tree form factor only
// usage: chol_bench <H file (NR*NR floats)> <rhs file (NR floats)> <mode> <nworld> <reps>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "engine_impl.h"
#include "chol_bench_dense.h"

using namespace mjx;
constexpr int NR = 36;

__global__ __launch_bounds__(64) void kbench(const float* Hg, const float* bg, float* xout,
                                             unsigned long long* cyc, int reps, int mode) {
  __shared__ float Hm[NR * NR];
  __shared__ float Lm[NR * NR];
  __shared__ float cb[4 * 64];
  const int lane = threadIdx.x;
  for (int i = lane; i < NR * NR; i += 64) Hm[i] = Hg[i];
  float b = lane < NR ? bg[lane] : 0.f;
  sync();
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  float x = 0.f;
  for (int r = 0; r < reps; r++) {
    float A[NR];
    float rd;
    rows_load<NR>(A, Hm, NR, lane);
    if (mode == 1) {
      old_rows_chol<NR>(A, rd, cb, NR, lane);
      old_rows_store_strict<NR>(A, rd, Lm, NR, lane);
      old_rows_fwd_rows<NR>(A, rd, lane);
      sync();
      x = old_rows_solve<NR>(A, rd, Lm, b + x * 1e-30f, NR, lane);
    } else if (mode == 6 || mode == 7) {  // tree form (reversed order), G1 dof tree (spec 1)
      rows_load_rev<NR>(A, Hm, NR, lane);
      rows_chol_tree<NR, 1>(A, rd, cb, lane);
      rows_store_strict<NR>(A, rd, Lm, NR, lane);
      if (mode == 7) {
        x += rd;
      } else {
        rows_fwd_rows<NR>(A, rd, lane);
        sync();
        const float bp = lane < NR ? __shfl(b, NR - 1 - lane) : 0.f;
        const float xp = rows_solve<NR>(A, rd, Lm, bp + x * 1e-30f, NR, lane);
        x = __shfl(xp, lane < NR ? NR - 1 - lane : lane);
      }
    } else if (mode == 5) {  // latency form: trailing reads a group ahead
      rows_chol<NR, true>(A, rd, cb, NR, lane);
      rows_store_strict<NR>(A, rd, Lm, NR, lane);
      x += rd;
    } else if (mode == 3) {  // factor only
      rows_chol<NR>(A, rd, cb, NR, lane);
      rows_store_strict<NR>(A, rd, Lm, NR, lane);
      x += rd;
    } else if (mode == 4) {  // solve only (factor of the first rep reused)
      if (r == 0) {
        rows_chol<NR>(A, rd, cb, NR, lane);
        rows_store_strict<NR>(A, rd, Lm, NR, lane);
        sync();
      }
      rows_load_factor<NR>(A, rd, Lm, NR, lane);
      x = rows_solve<NR>(A, rd, Lm, b + x * 1e-30f, NR, lane);
    } else {
      rows_chol<NR>(A, rd, cb, NR, lane);
      rows_store_strict<NR>(A, rd, Lm, NR, lane);
      rows_fwd_rows<NR>(A, rd, lane);
      sync();
      x = rows_solve<NR>(A, rd, Lm, b + x * 1e-30f, NR, lane);
    }
    sync();
  }
  __builtin_amdgcn_s_waitcnt(0);
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (lane < NR) xout[blockIdx.x * NR + lane] = x;
  if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

int main(int argc, char** argv) {
  if (argc < 6) { fprintf(stderr, "usage\n"); return 2; }
  std::vector<float> H(NR * NR), bv(NR);
  FILE* f = fopen(argv[1], "rb"); if (!f || fread(H.data(), 4, NR * NR, f) != NR * NR) return 2; fclose(f);
  f = fopen(argv[2], "rb"); if (!f || fread(bv.data(), 4, NR, f) != NR) return 2; fclose(f);
  const int mode = atoi(argv[3]), nw = atoi(argv[4]), reps = atoi(argv[5]);
  float *dH, *db, *dx; unsigned long long* dc;
  hipMalloc(&dH, 4 * NR * NR); hipMalloc(&db, 4 * NR); hipMalloc(&dx, 4 * NR * nw); hipMalloc(&dc, 8 * nw);
  hipMemcpy(dH, H.data(), 4 * NR * NR, hipMemcpyHostToDevice);
  hipMemcpy(db, bv.data(), 4 * NR, hipMemcpyHostToDevice);
  for (int it = 0; it < 3; it++) hipLaunchKernelGGL(kbench, dim3(nw), dim3(64), 0, 0, dH, db, dx, dc, reps, mode);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(kbench, dim3(nw), dim3(64), 0, 0, dH, db, dx, dc, reps, mode);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  std::vector<unsigned long long> c(nw); std::vector<float> x(NR);
  hipMemcpy(c.data(), dc, 8 * nw, hipMemcpyDeviceToHost);
  hipMemcpy(x.data(), dx, 4 * NR, hipMemcpyDeviceToHost);
  double mean = 0, mx = 0;
  for (auto v : c) { mean += v; mx = v > mx ? v : mx; }
  mean /= nw;
  printf("mode %d nworld %d: %.0f cycles/rep mean, %.0f max, kernel %.2f us/rep; x[0..3] %.6g %.6g %.6g %.6g\n",
         mode, nw, mean / reps, mx / reps, 1e3 * ms / reps, x[0], x[1], x[2], x[3]);
  f = fopen("gpurun_out/chol_x.bin", mode == 0 ? "wb" : "ab"); if (f) { fwrite(x.data(), 4, NR, f); fclose(f); }
  return 0;
}
