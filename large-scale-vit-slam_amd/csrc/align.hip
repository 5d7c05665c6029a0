// Point-map Sim(3) alignment on the GPU (include/vggt_mi355x.h:
// vggt_irls_sim3, vggt_sim3_points, vggt_scale_f32).
//
// vggt_irls_sim3 restates irls_sim3_umeyama + weighted_umeyama_sim3
// (aligned_vggt/models/pointAligned_wrapped_vggt.py:159-305) as a fixed
// sequence of launches with all state in device memory -- no host sync, no
// .item():
//   * combined confidence c = sqrt(conf_src * conf_dst); its lower median
//     (torch.median) by an exact 4-pass radix select over the float bits
//     (c >= 0, so the bit pattern orders like the value); points with
//     c < 0.5 * median get weight 0 (= the reference's boolean-mask filter);
//   * each weighted Umeyama solve = two grid-wide passes (weighted centroids,
//     then centred covariance + source variance) with per-block partial sums
//     reduced in a fixed order in fp64, and one single-thread solve: 3x3 SVD
//     via Jacobi on Sigma^T Sigma in fp64, R = U diag(1,1,sign det(UV^T)) V^T,
//     s = trace(S D) / var_x, t = mu_y - s R mu_x, rounded to fp32 (the
//     reference's dtype);
//   * IRLS: weights c * huber(|s R x + t - y|, delta) recomputed on the fly
//     from the previous iterate (fp32, as the reference), convergence when
//     |dR|_F, |dt|, |ds| < tol; later launches see the done flag and return.
// Every pass streams src/dst/conf (32 B per point) -- HBM-bound.
#include <math.h>

#include "common.h"

namespace {

constexpr int NB = 256;   // blocks per batch element in the reduction passes
constexpr int NTH = 256;  // threads per block

struct IrlsState {
  uint32_t prefix, pmask;  // radix-select prefix and mask of decided bits
  int64_t krank;           // remaining rank inside the current bucket
  float thr;               // 0.5 * median(c)
  int done, iters, err;
  float R[9], t[3], s;     // current iterate (fp32, the reference's dtype)
  double mux[3], muy[3], wsum;
};

struct IrlsArgs {
  const float *src, *dst, *cs, *cd;
  int64_t src_bs, dst_bs, cs_bs, cd_bs;  // batch strides (elements)
  int64_t n;                             // points per batch element
  float factor, delta, tol;
  IrlsState* st;    // [B]
  double* part;     // [B][NB][10]
  uint32_t* hist;   // [B][256]
  float *R_out, *t_out, *s_out;
};

// combined confidence; conf_dst == NULL: conf_src are the weights themselves
// (weighted_umeyama_sim3 called directly)
__device__ __forceinline__ float comb_at(const IrlsArgs& a, int b, int64_t i) {
  return a.cd ? sqrtf(a.cs[b * a.cs_bs + i] * a.cd[b * a.cd_bs + i]) : a.cs[b * a.cs_bs + i];
}

// ---- radix select of the lower median of c, one 8-bit digit per pass
__global__ __launch_bounds__(NTH) void irls_hist(IrlsArgs a, int pass) {
  __shared__ uint32_t h[256];
  const int b = blockIdx.y;
  const IrlsState& st = a.st[b];
  for (int i = threadIdx.x; i < 256; i += NTH) h[i] = 0;
  __syncthreads();
  const int shift = 24 - 8 * pass;
  for (int64_t i = blockIdx.x * (int64_t)NTH + threadIdx.x; i < a.n; i += (int64_t)gridDim.x * NTH) {
    const uint32_t u = __float_as_uint(comb_at(a, b, i));
    if ((u & st.pmask) == st.prefix) atomicAdd(&h[(u >> shift) & 255u], 1u);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 256; i += NTH)
    if (h[i]) atomicAdd(&a.hist[b * 256 + i], h[i]);
}

__global__ void irls_select(IrlsArgs a, int pass) {
  const int b = blockIdx.x;
  IrlsState& st = a.st[b];
  uint32_t* hb = a.hist + b * 256;
  if (threadIdx.x == 0) {
    const int shift = 24 - 8 * pass;
    int64_t k = st.krank, acc = 0;
    int d = 255;
    for (int i = 0; i < 256; ++i) {
      if (acc + hb[i] > k) {
        d = i;
        break;
      }
      acc += hb[i];
    }
    st.krank = k - acc;
    st.prefix |= (uint32_t)d << shift;
    st.pmask |= 255u << shift;
    if (pass == 3) st.thr = a.factor * __uint_as_float(st.prefix);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 256; i += blockDim.x) hb[i] = 0;  // ready for the next pass
}

// IRLS weight of point i under the current iterate (iteration 0: the
// combined confidence alone).
__device__ __forceinline__ float weight_at(const IrlsArgs& a, const IrlsState& st, int b, int64_t i, bool robust,
                                           float x0, float x1, float x2, float y0, float y1, float y2) {
  const float c = comb_at(a, b, i);
  if (!(c >= st.thr)) return 0.f;
  if (!robust) return c;
  // transformed = s * (src @ R^T) + t  (fp32)
  const float p0 = st.s * (x0 * st.R[0] + x1 * st.R[1] + x2 * st.R[2]) + st.t[0];
  const float p1 = st.s * (x0 * st.R[3] + x1 * st.R[4] + x2 * st.R[5]) + st.t[1];
  const float p2 = st.s * (x0 * st.R[6] + x1 * st.R[7] + x2 * st.R[8]) + st.t[2];
  const float d0 = p0 - y0, d1 = p1 - y1, d2 = p2 - y2;
  const float r = sqrtf(d0 * d0 + d1 * d1 + d2 * d2);
  return c * (r <= a.delta ? 1.f : a.delta / fmaxf(r, 1e-12f));
}

__device__ __forceinline__ double block_sum(double v, double* sh) {
  v = v + __shfl_xor(v, 32, 64);
  v = v + __shfl_xor(v, 16, 64);
  v = v + __shfl_xor(v, 8, 64);
  v = v + __shfl_xor(v, 4, 64);
  v = v + __shfl_xor(v, 2, 64);
  v = v + __shfl_xor(v, 1, 64);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sh[w] = v;
  __syncthreads();
  double s = 0.0;
  for (int i = 0; i < NTH / 64; ++i) s += sh[i];
  return s;
}

// pass 1: sum w, sum w x, sum w y
__global__ __launch_bounds__(NTH) void irls_pass1(IrlsArgs a, int robust) {
  __shared__ double sh[NTH / 64];
  const int b = blockIdx.y;
  const IrlsState& st = a.st[b];
  if (st.done) return;
  double acc[7] = {0, 0, 0, 0, 0, 0, 0};
  const float* x = a.src + b * a.src_bs;
  const float* y = a.dst + b * a.dst_bs;
  for (int64_t i = blockIdx.x * (int64_t)NTH + threadIdx.x; i < a.n; i += (int64_t)gridDim.x * NTH) {
    const float x0 = x[3 * i], x1 = x[3 * i + 1], x2 = x[3 * i + 2];
    const float y0 = y[3 * i], y1 = y[3 * i + 1], y2 = y[3 * i + 2];
    const double w = weight_at(a, st, b, i, robust, x0, x1, x2, y0, y1, y2);
    acc[0] += w;
    acc[1] += w * x0;
    acc[2] += w * x1;
    acc[3] += w * x2;
    acc[4] += w * y0;
    acc[5] += w * y1;
    acc[6] += w * y2;
  }
  double* out = a.part + ((int64_t)b * NB + blockIdx.x) * 10;
  for (int j = 0; j < 7; ++j) {
    const double s = block_sum(acc[j], sh);
    if (threadIdx.x == 0) out[j] = s;
  }
}

// pass 2: centroids (every block reduces pass 1's partials in the same fixed
// order), then sum w y_c x_c^T and sum w |x_c|^2
__global__ __launch_bounds__(NTH) void irls_pass2(IrlsArgs a, int robust) {
  __shared__ double sh[NTH / 64];
  __shared__ double mu[7];
  const int b = blockIdx.y;
  const IrlsState& st = a.st[b];
  if (st.done) return;
  if (threadIdx.x < 7) {
    double s = 0.0;
    const double* p = a.part + (int64_t)b * NB * 10 + threadIdx.x;
    for (int k = 0; k < NB; ++k) s += p[k * 10];
    mu[threadIdx.x] = s;
  }
  __syncthreads();
  const double W = mu[0];
  const double mx0 = mu[1] / W, mx1 = mu[2] / W, mx2 = mu[3] / W;
  const double my0 = mu[4] / W, my1 = mu[5] / W, my2 = mu[6] / W;
  double acc[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  const float* x = a.src + b * a.src_bs;
  const float* y = a.dst + b * a.dst_bs;
  for (int64_t i = blockIdx.x * (int64_t)NTH + threadIdx.x; i < a.n; i += (int64_t)gridDim.x * NTH) {
    const float x0 = x[3 * i], x1 = x[3 * i + 1], x2 = x[3 * i + 2];
    const float y0 = y[3 * i], y1 = y[3 * i + 1], y2 = y[3 * i + 2];
    const double w = weight_at(a, st, b, i, robust, x0, x1, x2, y0, y1, y2);
    const double cx0 = x0 - mx0, cx1 = x1 - mx1, cx2 = x2 - mx2;
    const double wy0 = w * (y0 - my0), wy1 = w * (y1 - my1), wy2 = w * (y2 - my2);
    acc[0] += wy0 * cx0;
    acc[1] += wy0 * cx1;
    acc[2] += wy0 * cx2;
    acc[3] += wy1 * cx0;
    acc[4] += wy1 * cx1;
    acc[5] += wy1 * cx2;
    acc[6] += wy2 * cx0;
    acc[7] += wy2 * cx1;
    acc[8] += wy2 * cx2;
    acc[9] += w * (cx0 * cx0 + cx1 * cx1 + cx2 * cx2);
  }
  __syncthreads();
  // (pass-1 partials are re-read by the solve below: keep them; write ours
  // after them in a second half of the scratch row block)
  double* out = a.part + ((int64_t)gridDim.y * NB + (int64_t)b * NB + blockIdx.x) * 10;
  for (int j = 0; j < 10; ++j) {
    const double s = block_sum(acc[j], sh);
    if (threadIdx.x == 0) out[j] = s;
  }
}

// ---- 3x3 symmetric eigen-decomposition (cyclic Jacobi, fp64)
__device__ void jacobi3(double A[3][3], double V[3][3]) {
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) V[i][j] = i == j ? 1.0 : 0.0;
  for (int sweep = 0; sweep < 32; ++sweep) {
    const double off = fabs(A[0][1]) + fabs(A[0][2]) + fabs(A[1][2]);
    const double scale = fabs(A[0][0]) + fabs(A[1][1]) + fabs(A[2][2]);
    if (off <= 1e-300 || off <= 1e-18 * scale) break;
    for (int p = 0; p < 2; ++p)
      for (int q = p + 1; q < 3; ++q) {
        if (A[p][q] == 0.0) continue;
        const double theta = (A[q][q] - A[p][p]) / (2.0 * A[p][q]);
        const double tt = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
        const double c = 1.0 / sqrt(tt * tt + 1.0), s = tt * c;
        for (int k = 0; k < 3; ++k) {  // A = J^T A J
          const double akp = A[k][p], akq = A[k][q];
          A[k][p] = c * akp - s * akq;
          A[k][q] = s * akp + c * akq;
        }
        for (int k = 0; k < 3; ++k) {
          const double apk = A[p][k], aqk = A[q][k];
          A[p][k] = c * apk - s * aqk;
          A[q][k] = s * apk + c * aqk;
        }
        for (int k = 0; k < 3; ++k) {
          const double vkp = V[k][p], vkq = V[k][q];
          V[k][p] = c * vkp - s * vkq;
          V[k][q] = s * vkp + c * vkq;
        }
      }
  }
}

__device__ __forceinline__ double det3(const double M[3][3]) {
  return M[0][0] * (M[1][1] * M[2][2] - M[1][2] * M[2][1]) - M[0][1] * (M[1][0] * M[2][2] - M[1][2] * M[2][0]) +
         M[0][2] * (M[1][0] * M[2][1] - M[1][1] * M[2][0]);
}

// weighted Umeyama closed form from the reduced sums (pointAligned :159-219)
__global__ void irls_solve(IrlsArgs a, int iter, int max_iters) {
  const int b = blockIdx.x;
  IrlsState& st = a.st[b];
  if (st.done || threadIdx.x != 0) return;
  double s1[7] = {0, 0, 0, 0, 0, 0, 0}, s2[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  const double* p1 = a.part + (int64_t)b * NB * 10;
  const double* p2 = a.part + ((int64_t)gridDim.x * NB + (int64_t)b * NB) * 10;
  for (int k = 0; k < NB; ++k) {
    for (int j = 0; j < 7; ++j) s1[j] += p1[k * 10 + j];
    for (int j = 0; j < 10; ++j) s2[j] += p2[k * 10 + j];
  }
  const double W = s1[0];
  if (W < 1e-6) {  // the reference raises ValueError("Total weight too small ...")
    st.err = 1;
    st.done = 1;
    for (int j = 0; j < 9; ++j) a.R_out[b * 9 + j] = NAN;
    for (int j = 0; j < 3; ++j) a.t_out[b * 3 + j] = NAN;
    a.s_out[b] = NAN;
    return;
  }
  const double mux[3] = {s1[1] / W, s1[2] / W, s1[3] / W};
  const double muy[3] = {s1[4] / W, s1[5] / W, s1[6] / W};
  double Sg[3][3];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) Sg[i][j] = s2[3 * i + j] / W;
  const double varx = s2[9] / W;
  // SVD Sg = U diag(sv) V^T via the eigen-decomposition of Sg^T Sg
  double A[3][3], V[3][3];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) A[i][j] = Sg[0][i] * Sg[0][j] + Sg[1][i] * Sg[1][j] + Sg[2][i] * Sg[2][j];
  jacobi3(A, V);
  int ord[3] = {0, 1, 2};  // eigenvalues descending
  for (int i = 0; i < 2; ++i)
    for (int j = 0; j < 2 - i; ++j)
      if (A[ord[j]][ord[j]] < A[ord[j + 1]][ord[j + 1]]) {
        const int tmp = ord[j];
        ord[j] = ord[j + 1];
        ord[j + 1] = tmp;
      }
  double Vs[3][3], U[3][3], sv[3];
  for (int k = 0; k < 3; ++k) {
    for (int i = 0; i < 3; ++i) Vs[i][k] = V[i][ord[k]];
  }
  // u_k = Sg v_k / |Sg v_k| for the two largest; u_2 = u_0 x u_1, and v_2's
  // sign chosen so that Sg v_2 = sv_2 u_2 with sv_2 >= 0 (a valid SVD pair)
  for (int k = 0; k < 2; ++k) {
    double u[3], nrm = 0.0;
    for (int i = 0; i < 3; ++i) {
      u[i] = Sg[i][0] * Vs[0][k] + Sg[i][1] * Vs[1][k] + Sg[i][2] * Vs[2][k];
      nrm += u[i] * u[i];
    }
    nrm = sqrt(nrm);
    sv[k] = nrm;
    for (int i = 0; i < 3; ++i) U[i][k] = nrm > 0 ? u[i] / nrm : (i == k ? 1.0 : 0.0);
  }
  U[0][2] = U[1][0] * U[2][1] - U[2][0] * U[1][1];
  U[1][2] = U[2][0] * U[0][1] - U[0][0] * U[2][1];
  U[2][2] = U[0][0] * U[1][1] - U[1][0] * U[0][1];
  {
    double u[3];
    for (int i = 0; i < 3; ++i) u[i] = Sg[i][0] * Vs[0][2] + Sg[i][1] * Vs[1][2] + Sg[i][2] * Vs[2][2];
    const double proj = u[0] * U[0][2] + u[1] * U[1][2] + u[2] * U[2][2];
    if (proj < 0) {
      for (int i = 0; i < 3; ++i) Vs[i][2] = -Vs[i][2];
    }
    sv[2] = fabs(proj);
  }
  // D = diag(1, 1, sign(det(U V^T)))
  double UVt[3][3];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) UVt[i][j] = U[i][0] * Vs[j][0] + U[i][1] * Vs[j][1] + U[i][2] * Vs[j][2];
  const double dt = det3(UVt);
  const double d = dt > 0 ? 1.0 : (dt < 0 ? -1.0 : 0.0);
  double R[3][3];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) R[i][j] = U[i][0] * Vs[j][0] + U[i][1] * Vs[j][1] + d * U[i][2] * Vs[j][2];
  const double s = (sv[0] + sv[1] + d * sv[2]) / varx;
  double t[3];
  for (int i = 0; i < 3; ++i) t[i] = muy[i] - s * (R[i][0] * mux[0] + R[i][1] * mux[1] + R[i][2] * mux[2]);
  // round to the reference dtype; convergence test against the previous iterate
  float Rf[9], tf[3];
  for (int i = 0; i < 9; ++i) Rf[i] = (float)R[i / 3][i % 3];
  for (int i = 0; i < 3; ++i) tf[i] = (float)t[i];
  const float sf = (float)s;
  bool conv = false;
  if (iter >= 1) {
    double dR = 0, dT = 0;
    for (int i = 0; i < 9; ++i) dR += (double)(Rf[i] - st.R[i]) * (double)(Rf[i] - st.R[i]);
    for (int i = 0; i < 3; ++i) dT += (double)(tf[i] - st.t[i]) * (double)(tf[i] - st.t[i]);
    conv = sqrt(dR) < a.tol && sqrt(dT) < a.tol && fabs((double)(sf - st.s)) < a.tol;
  }
  for (int i = 0; i < 9; ++i) st.R[i] = Rf[i];
  for (int i = 0; i < 3; ++i) st.t[i] = tf[i];
  st.s = sf;
  st.iters = iter;
  for (int i = 0; i < 9; ++i) a.R_out[b * 9 + i] = Rf[i];
  for (int i = 0; i < 3; ++i) a.t_out[b * 3 + i] = tf[i];
  a.s_out[b] = sf;
  if (conv || iter >= max_iters) st.done = 1;
}

__global__ void irls_reset(IrlsArgs a) {
  const int b = blockIdx.x;
  IrlsState& st = a.st[b];
  if (threadIdx.x == 0) {
    st.prefix = 0;
    st.pmask = 0;
    st.krank = (a.n - 1) / 2;  // torch.median: the lower of the two middle values
    st.thr = 0.f;
    st.done = 0;
    st.iters = 0;
    st.err = 0;
  }
  for (int i = threadIdx.x; i < 256; i += blockDim.x) a.hist[b * 256 + i] = 0;
}

// ---- dense Sim(3) application: out = T[:3,:3] (s p) + T[:3,3]
// (apply_sim3_alignment_on_point_maps, alignment.py:491-526)
__global__ __launch_bounds__(256) void sim3_points_kernel(const float* __restrict__ p, int64_t p_bs, int64_t n,
                                                          const float* __restrict__ T, const float* __restrict__ sc,
                                                          float* __restrict__ out, int64_t o_bs) {
  const int b = blockIdx.y;
  const float* Tb = T + b * 16;
  const float s = sc ? sc[b] : 1.f;
  const float r00 = Tb[0], r01 = Tb[1], r02 = Tb[2], t0 = Tb[3];
  const float r10 = Tb[4], r11 = Tb[5], r12 = Tb[6], t1 = Tb[7];
  const float r20 = Tb[8], r21 = Tb[9], r22 = Tb[10], t2 = Tb[11];
  const float* pb = p + b * p_bs;
  float* ob = out + b * o_bs;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float x = pb[3 * i] * s, y = pb[3 * i + 1] * s, z = pb[3 * i + 2] * s;
    ob[3 * i] = r00 * x + r01 * y + r02 * z + t0;
    ob[3 * i + 1] = r10 * x + r11 * y + r12 * z + t1;
    ob[3 * i + 2] = r20 * x + r21 * y + r22 * z + t2;
  }
}

__global__ __launch_bounds__(256) void scale_kernel(float* __restrict__ x, int64_t bs, int64_t n,
                                                    const float* __restrict__ sc) {
  const int b = blockIdx.y;
  const float s = sc[b];
  float* xb = x + b * bs;
  const int64_t n4 = ((bs & 3) == 0 && ((uintptr_t)x & 15) == 0) ? n / 4 : 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    f32x4 v = ((f32x4*)xb)[i];
    v *= s;
    ((f32x4*)xb)[i] = v;
  }
  for (int64_t i = 4 * n4 + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    xb[i] *= s;
}

}  // namespace

extern "C" size_t vggt_irls_workspace_bytes(int B) {
  return (size_t)B * sizeof(IrlsState) + (size_t)2 * B * NB * 10 * sizeof(double) + (size_t)B * 256 * 4 + 256;
}

extern "C" int vggt_irls_sim3(const float* src, int64_t src_bs, const float* dst, int64_t dst_bs, const float* conf_src,
                              int64_t cs_bs, const float* conf_dst, int64_t cd_bs, int B, int64_t n, float factor,
                              float delta, int max_iters, float tol, float* R_out, float* t_out, float* s_out,
                              void* workspace, size_t ws_bytes, void* stream) {
  if (B <= 0 || n <= 0 || max_iters < 0) return VGGT_ERR_SHAPE;
  if (ws_bytes < vggt_irls_workspace_bytes(B) || ((uintptr_t)workspace & 15)) return VGGT_ERR_ALIGN;
  char* ws = (char*)workspace;
  IrlsArgs a;
  a.src = src;
  a.dst = dst;
  a.cs = conf_src;
  a.cd = conf_dst;
  a.src_bs = src_bs;
  a.dst_bs = dst_bs;
  a.cs_bs = cs_bs;
  a.cd_bs = cd_bs;
  a.n = n;
  a.factor = factor;
  a.delta = delta;
  a.tol = tol;
  a.part = (double*)ws;
  ws += (size_t)2 * B * NB * 10 * sizeof(double);
  a.st = (IrlsState*)ws;
  ws += ((size_t)B * sizeof(IrlsState) + 15) & ~(size_t)15;
  a.hist = (uint32_t*)ws;
  a.R_out = R_out;
  a.t_out = t_out;
  a.s_out = s_out;
  hipStream_t s = (hipStream_t)stream;
  irls_reset<<<B, 256, 0, s>>>(a);
  if (factor > 0.f) {  // factor <= 0: no confidence threshold (thr stays 0, weights >= 0 all kept)
    const int hblocks = (int)((n + NTH - 1) / NTH < 1024 ? (n + NTH - 1) / NTH : 1024);
    for (int pass = 0; pass < 4; ++pass) {
      irls_hist<<<dim3(hblocks, B), NTH, 0, s>>>(a, pass);
      irls_select<<<B, 256, 0, s>>>(a, pass);
    }
  }
  for (int it = 0; it <= max_iters; ++it) {  // it = 0: the initial solve on the confidences alone
    irls_pass1<<<dim3(NB, B), NTH, 0, s>>>(a, it > 0);
    irls_pass2<<<dim3(NB, B), NTH, 0, s>>>(a, it > 0);
    irls_solve<<<B, 64, 0, s>>>(a, it, max_iters);
  }
  HIP_LAUNCH_CHECK();
  return VGGT_OK;
}

extern "C" int vggt_sim3_points(const float* pts, int64_t p_bs, int B, int64_t n, const float* T, const float* scale,
                                float* out, int64_t o_bs, void* stream) {
  if (B <= 0 || n < 0) return VGGT_ERR_SHAPE;
  if (n == 0) return VGGT_OK;
  const int64_t blocks = (n + 255) / 256;
  sim3_points_kernel<<<dim3((unsigned)(blocks < 2048 ? blocks : 2048), B), 256, 0, (hipStream_t)stream>>>(
      pts, p_bs, n, T, scale, out, o_bs);
  HIP_LAUNCH_CHECK();
  return VGGT_OK;
}

extern "C" int vggt_scale_f32(float* x, int64_t bs, int B, int64_t n, const float* scale, void* stream) {
  if (B <= 0 || n < 0) return VGGT_ERR_SHAPE;
  if (n == 0) return VGGT_OK;
  const int64_t blocks = (n / 4 + 255) / 256 + 1;
  scale_kernel<<<dim3((unsigned)(blocks < 2048 ? blocks : 2048), B), 256, 0, (hipStream_t)stream>>>(x, bs, n, scale);
  HIP_LAUNCH_CHECK();
  return VGGT_OK;
}
