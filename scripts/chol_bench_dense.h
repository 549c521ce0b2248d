// Pre-round-3 register-row SPD forms, kept for the chol_bench A/B only.
#pragma once
namespace mjx {
template <int NR>
__device__ __forceinline__ void old_rows_load(float (&A)[NR], const float* Mm, int nvp, int lane) {
  const int row = lane < nvp ? lane : 0;
#pragma unroll
  for (int c = 0; c < NR; c += 4) {
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (c < nvp) v = ld4(Mm + row * nvp + c);
    A[c] = v.x; A[c + 1] = v.y; A[c + 2] = v.z; A[c + 3] = v.w;
  }
  if (lane >= nvp) {
#pragma unroll
    for (int c = 0; c < NR; c++) A[c] = c == lane ? 1.f : 0.f;
  }
}
// In-place blocked right-looking Cholesky of the lower triangle: afterwards A[c] (c <= lane)
// is L[lane][c] and rdiag = 1/L[lane][lane].  Entries above the diagonal are scratch; they
// never feed the lower part.  Columns go in blocks of 4: the diagonal block is factored with
// v_readlane broadcasts (6 per block), then each lane publishes its 4 block entries to
// `cb` (LDS, 4*64 floats: every lane writes, no branch) and every lane reads the block rows of the trailing columns back
// as broadcast float4s -- one LDS round trip per 4 columns instead of one v_readlane per
// trailing element (630 for NR 36).
template <int NR>
__device__ __forceinline__ void old_rows_chol(float (&A)[NR], float& rdiag, float* cb, int nvp, int lane) {
  static_assert(NR % 4 == 0, "register rows come in column blocks of 4");
  rdiag = 1.f;
  // Padding rows/cols (>= nvp) are identity/zero, so the full NR sweep is exact there:
  // no per-step guards (guards get hoisted into spilled SGPR masks).
#pragma unroll
  for (int j0 = 0; j0 < NR; j0 += 4) {
#pragma unroll
    for (int t = 0; t < 4; t++) {
      const int j = j0 + t;
      const float r = __builtin_amdgcn_rsqf(fmaxf(rl(A[j], j), MINVAL));
      A[j] *= r;
      rdiag = lane == j ? r : rdiag;
#pragma unroll
      for (int u = t + 1; u < 4; u++) A[j0 + u] = fmaf(-A[j], rl(A[j], j0 + u), A[j0 + u]);
    }
    if (j0 + 4 < NR) {
      st4v(cb + 4 * lane, make_float4(A[j0], A[j0 + 1], A[j0 + 2], A[j0 + 3]));  // all 64 lanes (no branch)
      sync();
      // trailing columns in groups of 4 (at most 16 broadcast VGPRs in flight: unbounded,
      // the scheduler hoists every read of the block and the kernel loses occupancy)
#pragma unroll
      for (int k0 = j0 + 4; k0 < NR; k0 += 4) {
        float4 c[4];
#pragma unroll
        for (int u = 0; u < 4; u++) c[u] = ld4(cb + 4 * (k0 + u));  // row k of the block: broadcast
#pragma unroll
        for (int u = 0; u < 4; u++)
          A[k0 + u] = fmaf(-A[j0 + 3], c[u].w, fmaf(-A[j0 + 2], c[u].z,
                      fmaf(-A[j0 + 1], c[u].y, fmaf(-A[j0], c[u].x, A[k0 + u]))));
      }
      sync();  // the next block's publish follows these reads
    }
  }
  (void)nvp;
}
// The triangular solves run on scaled copies of L so that each of their 2*NR sequential
// steps is one v_readlane plus one FMA (no per-step rescale or select):
//   forward  L y = b   as u = diag(L) y:  u_j = b_j - sum_{k<j} M_jk u_k,  M_jk = L_jk / L_kk
//   backward L^T x = y as v = diag(L) x:  v_j = y_j - sum_{k>j} N_kj v_k,  N_kj = L_kj / L_kk
// M is column-scaled (register rows, rows_fwd_rows), N row-scaled (published to LDS by
// rows_store_strict and read back by columns).
// Publish N (row stride nvp): strictly-lower part, 1/L[i][i] on the diagonal, zeros above.
template <int NR>
__device__ __forceinline__ void old_rows_store_strict(const float (&A)[NR], float rd, float* Lm, int nvp,
                                                  int lane) {
  if (lane >= nvp) return;
#pragma unroll
  for (int c = 0; c < NR; c += 4)
    if (c < nvp)
      st4v(Lm + lane * nvp + c,
           make_float4(c < lane ? A[c] * rd : c == lane ? rd : 0.f,
                       c + 1 < lane ? A[c + 1] * rd : c + 1 == lane ? rd : 0.f,
                       c + 2 < lane ? A[c + 2] * rd : c + 2 == lane ? rd : 0.f,
                       c + 3 < lane ? A[c + 3] * rd : c + 3 == lane ? rd : 0.f));
}
// Factor rows L (rows_chol) -> forward rows M (strictly lower, column-scaled).
template <int NR>
__device__ __forceinline__ void old_rows_fwd_rows(float (&A)[NR], float rd, int lane) {
#pragma unroll
  for (int k = 0; k < NR; k++) A[k] = k < lane ? A[k] * rl(rd, k) : 0.f;
}
// Forward rows M of a factor published by rows_store_strict (M_jk = N_jk L_jj / L_kk), and
// this lane's 1/L[i][i].
template <int NR>
__device__ __forceinline__ void old_rows_load_factor(float (&A)[NR], float& rd, const float* Lm, int nvp,
                                                 int lane) {
  old_rows_load<NR>(A, Lm, nvp, lane);
  rd = lane < nvp ? Lm[lane * nvp + lane] : 1.f;
  const float ljj = __builtin_amdgcn_rcpf(rd);
#pragma unroll
  for (int k = 0; k < NR; k++) A[k] = k < lane ? A[k] * (rl(rd, k) * ljj) : 0.f;
}
// x (lane i holds x[i]) <- (L L^T)^-1 x, from the forward rows M (registers) and the columns
// of N in Lm (rows_store_strict, then synced).  Lanes >= nvp hold x = 0 and stay 0.
template <int NR>
__device__ __forceinline__ float old_rows_solve(const float (&M)[NR], float rdiag, const float* Lm,
                                            float x, int nvp, int lane) {
  float u = x;
#pragma unroll
  for (int j = 0; j < NR; j++) u = fmaf(-M[j], rl(u, j), u);  // M[j] = 0 on lanes <= j
  float Nc[NR];
  const int col = lane < nvp ? lane : 0;
#pragma unroll
  for (int j = 0; j < NR; j++) Nc[j] = (j < nvp && j > lane) ? Lm[j * nvp + col] : 0.f;
  float v = u * rdiag;  // y = u / L_jj: the backward sweep starts at v = y
#pragma unroll
  for (int j = NR - 1; j >= 0; j--) v = fmaf(-Nc[j], rl(v, j), v);
  return v * rdiag;
}
}  // namespace mjx
