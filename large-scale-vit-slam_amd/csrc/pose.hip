// Per-chunk pose / Sim(3) composition of FeatureAlignedVGGT.forward
// (featureAligned_vggt.py:96-143, 187-196) as one launch: the (B, S, 4, 4)
// SE(3) chain, the Markley quaternion mean over the overlap (geometry.py:4-37,
// a 4x4 symmetric eigenproblem solved by cyclic Jacobi on the device) and the
// final pose encoding -- no host round trip per chunk.
//
// One 64-lane workgroup per batch element; lane f (stride 64) owns frame f.
// All pose algebra in fp32 as the reference (autocast is disabled there,
// featureAligned_vggt.py:104); the Jacobi sweeps run in fp64 and the unit
// eigenvector is rounded to fp32 like torch.linalg.eigh's fp32 result (its
// sign is arbitrary in both, SURVEY Appendix A.7 -- and irrelevant here: the
// mean only enters through quat_to_mat, which is even in q).
#include "common.h"

namespace {

struct Aff {  // rows 0..2 of a 4x4 SE(3) / Sim(3) matrix, row 3 = (0, 0, 0, 1)
  float r[3][3];
  float t[3];
};

// VGGT rotation.quat_to_mat: scalar-last (x, y, z, w), 2 / |q|^2 scaling
__device__ void quat_to_mat(const float* q, float R[3][3]) {
  const float i = q[0], j = q[1], k = q[2], r = q[3];
  const float two_s = 2.0f / (q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  R[0][0] = 1.f - two_s * (j * j + k * k);
  R[0][1] = two_s * (i * j - k * r);
  R[0][2] = two_s * (i * k + j * r);
  R[1][0] = two_s * (i * j + k * r);
  R[1][1] = 1.f - two_s * (i * i + k * k);
  R[1][2] = two_s * (j * k - i * r);
  R[2][0] = two_s * (i * k - j * r);
  R[2][1] = two_s * (j * k + i * r);
  R[2][2] = 1.f - two_s * (i * i + j * j);
}

__device__ __forceinline__ float sqrt_pos(float x) { return x > 0.f ? sqrtf(x) : 0.f; }

// VGGT rotation.mat_to_quat: the best-conditioned of the four candidates,
// divided by 2 max(|q_i|, 0.1), reordered to (x, y, z, w), w >= 0
__device__ void mat_to_quat(const float R[3][3], float* q) {
  const float m00 = R[0][0], m01 = R[0][1], m02 = R[0][2], m10 = R[1][0], m11 = R[1][1], m12 = R[1][2],
              m20 = R[2][0], m21 = R[2][1], m22 = R[2][2];
  float qa[4] = {sqrt_pos(1.f + m00 + m11 + m22), sqrt_pos(1.f + m00 - m11 - m22), sqrt_pos(1.f - m00 + m11 - m22),
                 sqrt_pos(1.f - m00 - m11 + m22)};
  int b = 0;
  for (int i = 1; i < 4; ++i)
    if (qa[i] > qa[b]) b = i;  // first maximum, as torch.argmax
  float c[4];  // (w, x, y, z)
  switch (b) {
    case 0: c[0] = qa[0] * qa[0]; c[1] = m21 - m12; c[2] = m02 - m20; c[3] = m10 - m01; break;
    case 1: c[0] = m21 - m12; c[1] = qa[1] * qa[1]; c[2] = m10 + m01; c[3] = m02 + m20; break;
    case 2: c[0] = m02 - m20; c[1] = m10 + m01; c[2] = qa[2] * qa[2]; c[3] = m12 + m21; break;
    default: c[0] = m10 - m01; c[1] = m20 + m02; c[2] = m21 + m12; c[3] = qa[3] * qa[3]; break;
  }
  const float d = 2.0f * fmaxf(qa[b], 0.1f);
  float x = c[1] / d, y = c[2] / d, z = c[3] / d, w = c[0] / d;
  if (w < 0.f) { x = -x; y = -y; z = -z; w = -w; }
  q[0] = x; q[1] = y; q[2] = z; q[3] = w;
}

__device__ __forceinline__ void normalize4(float* q) {
  const float n = fmaxf(sqrtf(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]), 1e-8f);
  for (int i = 0; i < 4; ++i) q[i] = q[i] / n;
}

// aligned_vggt/utils/data.py:33-52: [T, quat] -> SE(3), quat normalised first
__device__ Aff enc_to_aff(const float* e) {
  float q[4] = {e[3], e[4], e[5], e[6]};
  normalize4(q);
  Aff a;
  quat_to_mat(q, a.r);
  a.t[0] = e[0]; a.t[1] = e[1]; a.t[2] = e[2];
  return a;
}

__device__ Aff mul(const Aff& a, const Aff& b) {  // a @ b
  Aff o;
  for (int i = 0; i < 3; ++i) {
    for (int j = 0; j < 3; ++j) o.r[i][j] = a.r[i][0] * b.r[0][j] + a.r[i][1] * b.r[1][j] + a.r[i][2] * b.r[2][j];
    o.t[i] = a.r[i][0] * b.t[0] + a.r[i][1] * b.t[1] + a.r[i][2] * b.t[2] + a.t[i];
  }
  return o;
}

// VGGT geometry.closed_form_inverse_se3: [R^T | -R^T t]
__device__ Aff inv_se3(const Aff& a) {
  Aff o;
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) o.r[i][j] = a.r[j][i];
  for (int i = 0; i < 3; ++i) o.t[i] = -(o.r[i][0] * a.t[0] + o.r[i][1] * a.t[1] + o.r[i][2] * a.t[2]);
  return o;
}

// Largest-eigenvalue unit eigenvector of a symmetric 4x4 (cyclic Jacobi, fp64).
__device__ void top_eigvec4(const double Min[4][4], double* v) {
  double A[4][4], V[4][4];
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j) {
      A[i][j] = Min[i][j];
      V[i][j] = i == j ? 1.0 : 0.0;
    }
  for (int sweep = 0; sweep < 32; ++sweep) {
    double off = 0.0;
    for (int p = 0; p < 4; ++p)
      for (int q = p + 1; q < 4; ++q) off += A[p][q] * A[p][q];
    if (off < 1e-60) break;
    for (int p = 0; p < 3; ++p)
      for (int q = p + 1; q < 4; ++q) {
        if (fabs(A[p][q]) < 1e-300) continue;
        const double theta = (A[q][q] - A[p][p]) / (2.0 * A[p][q]);
        const double t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
        const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
        for (int k = 0; k < 4; ++k) {  // A <- J^T A J
          const double akp = A[k][p], akq = A[k][q];
          A[k][p] = c * akp - s * akq;
          A[k][q] = s * akp + c * akq;
        }
        for (int k = 0; k < 4; ++k) {
          const double apk = A[p][k], aqk = A[q][k];
          A[p][k] = c * apk - s * aqk;
          A[q][k] = s * apk + c * aqk;
        }
        for (int k = 0; k < 4; ++k) {
          const double vkp = V[k][p], vkq = V[k][q];
          V[k][p] = c * vkp - s * vkq;
          V[k][q] = s * vkp + c * vkq;
        }
      }
  }
  int b = 0;
  for (int i = 1; i < 4; ++i)
    if (A[i][i] > A[b][b]) b = i;
  double n = 0.0;
  for (int k = 0; k < 4; ++k) n += V[k][b] * V[k][b];
  n = sqrt(n);
  for (int k = 0; k < 4; ++k) v[k] = V[k][b] / n;
}

constexpr int MAX_OV = 64;

__global__ __launch_bounds__(64) void pose_compose_kernel(
    const float* __restrict__ chunk_sim3, const float* __restrict__ frame_se3, const float* __restrict__ cam,
    const float* __restrict__ ctx, int S_prev, const float* __restrict__ gt_first, int S, int ov, float H, float W,
    float* __restrict__ out, float* __restrict__ pt_out) {
  const int b = blockIdx.x;
  const int lane = threadIdx.x;
  __shared__ Aff s_chunk, s_ident, s_mean, s_ptid;
  __shared__ float s_scale;
  __shared__ float s_ct[MAX_OV][7];  // overlap transforms as [t, quat] (Markley input)
  const float* cs = chunk_sim3 + (int64_t)b * 8;
  const float* cb = cam + (int64_t)b * S * 9;
  if (lane == 0) {
    s_chunk = enc_to_aff(cs);  // featureAligned_vggt.py:97
    s_scale = cs[7];           // :98
    // pose_encoding_to_extri_intri (VGGT): quat_to_mat on the raw quaternion
    Aff e0;
    quat_to_mat(cb + 3, e0.r);
    e0.t[0] = cb[0]; e0.t[1] = cb[1]; e0.t[2] = cb[2];
    s_ptid = e0;               // point_identity_alignment, :115
    s_ident = inv_se3(e0);     // :114
  }
  __syncthreads();
  // camera extrinsics of frame f: re-centred on frame 0, translation scaled (:109-119)
  auto extr = [&](int f) {
    const float* c = cb + (int64_t)f * 9;
    Aff e;
    quat_to_mat(c + 3, e.r);
    e.t[0] = c[0]; e.t[1] = c[1]; e.t[2] = c[2];
    e = mul(e, s_ident);
    for (int i = 0; i < 3; ++i) e.t[i] *= s_scale;
    return e;
  };
  // initial chunk alignment (:121-137)
  if (ctx == nullptr) {
    if (lane == 0) {
      Aff I;
      for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j) I.r[i][j] = i == j ? 1.f : 0.f;
        I.t[i] = 0.f;
      }
      s_mean = I;
    }
  } else if (gt_first != nullptr) {
    if (lane == 0) {
      const float* g = gt_first + (int64_t)b * 16;
      Aff m;
      for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j) m.r[i][j] = g[i * 4 + j];
        m.t[i] = g[i * 4 + 3];
      }
      s_mean = m;
    }
  } else {
    const float* cx = ctx + (int64_t)b * S_prev * 9;
    for (int k = lane; k < ov; k += 64) {
      const Aff co = enc_to_aff(cx + (int64_t)(S_prev - ov + k) * 9);  // context pose_enc[-1][:, -ov:], :126
      const Aff ct = mul(inv_se3(extr(k)), co);                      // :127-128
      if (ov == 1) {
        s_mean = ct;                                                   // :135
      } else {                                                         // extri_to_pose_encoding (data.py:12-30)
        float q[4];
        mat_to_quat(ct.r, q);
        normalize4(q);
        s_ct[k][0] = ct.t[0]; s_ct[k][1] = ct.t[1]; s_ct[k][2] = ct.t[2];
        for (int i = 0; i < 4; ++i) s_ct[k][3 + i] = q[i];
      }
    }
    __syncthreads();
    if (ov > 1 && lane == 0) {  // averagePoseEncodings (geometry.py:4-37)
      float t[3] = {0.f, 0.f, 0.f};
      for (int k = 0; k < ov; ++k)
        for (int i = 0; i < 3; ++i) t[i] += s_ct[k][i];
      const float inv_n = 1.0f / (float)ov;
      float M[4][4] = {};
      for (int k = 0; k < ov; ++k) {
        float q[4] = {s_ct[k][3], s_ct[k][4], s_ct[k][5], s_ct[k][6]};
        normalize4(q);
        for (int i = 0; i < 4; ++i)
          for (int j = 0; j < 4; ++j) M[i][j] += inv_n * (q[i] * q[j]);
      }
      double Md[4][4], v[4];
      for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) Md[i][j] = M[i][j];
      top_eigvec4(Md, v);
      float e[7] = {t[0] / (float)ov, t[1] / (float)ov, t[2] / (float)ov, (float)v[0], (float)v[1], (float)v[2],
                    (float)v[3]};
      s_mean = enc_to_aff(e);  // pose_encoding_to_extri(mean), :133
    }
  }
  __syncthreads();
  // per-frame SE(3) (:99-101), composed with the mean transform (:139) and the
  // camera extrinsics (:142), then encoded with the camera FoV (:143)
  const float* fb = frame_se3 + (int64_t)b * (S - 1) * 7;
  for (int f = lane; f < S; f += 64) {
    Aff pf = f == 0 ? s_chunk : mul(enc_to_aff(fb + (int64_t)(f - 1) * 7), s_chunk);
    pf = mul(pf, s_mean);
    const Aff a = mul(extr(f), pf);
    float q[4];
    mat_to_quat(a.r, q);
    const float* c = cb + (int64_t)f * 9;
    // pose_encoding_to_extri_intri -> intrinsics -> extri_intri_to_pose_encoding
    const float fy = (H / 2.0f) / tanf(c[7] / 2.0f);
    const float fx = (W / 2.0f) / tanf(c[8] / 2.0f);
    float* o = out + ((int64_t)b * S + f) * 9;
    o[0] = a.t[0]; o[1] = a.t[1]; o[2] = a.t[2];
    o[3] = q[0]; o[4] = q[1]; o[5] = q[2]; o[6] = q[3];
    o[7] = 2.0f * atanf((H / 2.0f) / fy);
    o[8] = 2.0f * atanf((W / 2.0f) / fx);
    if (f == 0 && pt_out != nullptr) {
      // point transform (:188-195): context ? inv(per_frame_se3[:, 0]) @ ptid : ptid
      const Aff p = ctx != nullptr ? mul(inv_se3(pf), s_ptid) : s_ptid;
      float* po = pt_out + (int64_t)b * 16;
      for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j) po[i * 4 + j] = p.r[i][j];
        po[i * 4 + 3] = p.t[i];
      }
      po[12] = 0.f; po[13] = 0.f; po[14] = 0.f; po[15] = 1.f;
    }
  }
}

}  // namespace

extern "C" int vggt_pose_compose(const float* chunk_sim3, const float* frame_se3, const float* cam_pose_enc,
                                 const float* ctx_pose_enc, int S_prev, const float* gt_first, int B, int S,
                                 int overlap, int H, int W, float* aligned_pose_enc, float* point_transform,
                                 void* stream) {
  if (B <= 0 || S <= 0 || H <= 0 || W <= 0) return VGGT_ERR_SHAPE;
  if (!chunk_sim3 || !cam_pose_enc || !aligned_pose_enc || (S > 1 && !frame_se3)) return VGGT_ERR_SHAPE;
  if (ctx_pose_enc != nullptr && gt_first == nullptr) {
    if (overlap < 1 || overlap > S || overlap > S_prev || overlap > MAX_OV) return VGGT_ERR_SHAPE;
  }
  pose_compose_kernel<<<B, 64, 0, (hipStream_t)stream>>>(chunk_sim3, frame_se3, cam_pose_enc, ctx_pose_enc, S_prev,
                                                         gt_first, S, overlap, (float)H, (float)W, aligned_pose_enc,
                                                         point_transform);
  HIP_LAUNCH_CHECK();
  return VGGT_OK;
}
