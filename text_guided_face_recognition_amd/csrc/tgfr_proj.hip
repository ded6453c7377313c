// Small-batch fp32 heads around the contrastive losses, exact fp32 FMA:
//
//   proj_fwd        g = normalize(x W^T + b) per row: the global projection
//                   head (ImageHeading.project_global, models/models.py:98-120
//                   and :336 -- Linear(512, 256) then F.normalize(dim = 1)).
//                   Block = (32 output columns, 8 rows); W's 32 rows and the 8
//                   x rows staged in LDS; each thread one output.  The row
//                   norms need every column group: the last block of each row
//                   group to finish (last_arrival) sums the groups' squares in
//                   group order and writes the normalised rows.
//   proj_dw         dW = dy^T x and db = colsum(dy) for the l2-norm backward's
//                   dy (tgfr_l2norm_rows_bwd), B <= 64: one launch, 256 blocks.
//   arc_dx_part     partial dxn = dcs W over class chunks (ArcMarginProduct's
//                   input side, models/metrics.py:43-44: dcs = dcos / |W_c|
//                   written by the ArcMargin backward)
//   arc_dx_finish   the chunks summed in chunk order, then the x l2-norm
//                   backward; one wave per row.
//
// These replace, per train step, split-bf16 GEMMs with their k-split reduces,
// an l2-norm, an l2-norm backward and the bias-gradient kernel (8 launches at
// B = 64) with 5.  The products are 8-75 M FMA: latency-bound chains of a few
// memory round trips, so every block issues all its loads at once, and the
// arithmetic is fp32 FMA on the VALU (exact products, fixed summation order).
#include "tgfr_common.h"

using namespace tgfr;

namespace {

constexpr int PJ_COLS = 32;     // output columns per forward block
constexpr int PJ_ROWS = 8;      // rows per forward block
constexpr int AD_ROWS = 16;     // rows per arc_dx_part block

// x [B][K] rows, W [N][K] (nn.Linear weight), y = x W^T + b.
// Block = (32 columns, 8 rows), 4 waves splitting K in quarters; lane =
// (row pair, column pair): per 4-k step 2 x + 2 W ds_read_b128 for 16 FMA.
// The staging loads of a block are all in flight at once (one L2 round trip).
// LDS: W slice [32][K + 4] | x rows [8][K + 4] | wave partials [4][256] | flag.
constexpr int PJ_STG = 24;      // float4 staging loads per thread (K <= 612)
__global__ __launch_bounds__(256) void proj_fwd_kernel(
    const float* __restrict__ x, long long ldx, int B, int K, const float* __restrict__ W,
    long long ldw, const float* __restrict__ bias, int N, float eps, float* __restrict__ yws,
    float* __restrict__ ssws, float* __restrict__ g, long long ldg, float* __restrict__ inv_norm,
    unsigned* __restrict__ counters) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int cg = blockIdx.x, rg = blockIdx.y;
  const int n0 = cg * PJ_COLS, r0 = rg * PJ_ROWS;
  const int P = K + 4;                                   // LDS row pitch (floats)
  float* ws = (float*)g_smem;
  float* xs = ws + PJ_COLS * P;
  float* red = xs + PJ_ROWS * P;
  int* flag = (int*)(red + 4 * 256);
  const int K4 = K / 4;
  const int items = (PJ_COLS + PJ_ROWS) * K4;
  {
    float4 v[PJ_STG];
#pragma unroll
    for (int u = 0; u < PJ_STG; ++u) {
      const int i = u * 256 + tid;
      v[u] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (i < items) {
        const int row = i / K4, c4 = i % K4;
        if (row < PJ_COLS)
          v[u] = *(const float4*)(W + (long long)(n0 + row) * ldw + 4 * c4);
        else if (r0 + row - PJ_COLS < B)
          v[u] = *(const float4*)(x + (long long)(r0 + row - PJ_COLS) * ldx + 4 * c4);
      }
    }
#pragma unroll
    for (int u = 0; u < PJ_STG; ++u) {
      const int i = u * 256 + tid;
      if (i < items) {
        const int row = i / K4, c4 = i % K4;
        *(float4*)(ws + row * P + 4 * c4) = v[u];    // x rows follow W's in LDS
      }
    }
  }
  __syncthreads();
  // wave w: k in [kq0, kq1) (4-k steps); lane: rows 2 rp, 2 rp + 1, columns 2 cp, 2 cp + 1
  const int rp = lane >> 4, cp = lane & 15;
  const int kq0 = w * K4 / 4, kq1 = (w + 1) * K4 / 4;
  const float* x0 = xs + (2 * rp) * P;
  const float* x1 = x0 + P;
  const float* w0 = ws + (2 * cp) * P;
  const float* w1 = w0 + P;
  float a00 = 0.f, a01 = 0.f, a10 = 0.f, a11 = 0.f;
  for (int kq = kq0; kq < kq1; ++kq) {
    const float4 xa = *(const float4*)(x0 + 4 * kq), xb = *(const float4*)(x1 + 4 * kq);
    const float4 wa = *(const float4*)(w0 + 4 * kq), wb = *(const float4*)(w1 + 4 * kq);
    a00 = fmaf(xa.x, wa.x, fmaf(xa.y, wa.y, fmaf(xa.z, wa.z, fmaf(xa.w, wa.w, a00))));
    a01 = fmaf(xa.x, wb.x, fmaf(xa.y, wb.y, fmaf(xa.z, wb.z, fmaf(xa.w, wb.w, a01))));
    a10 = fmaf(xb.x, wa.x, fmaf(xb.y, wa.y, fmaf(xb.z, wa.z, fmaf(xb.w, wa.w, a10))));
    a11 = fmaf(xb.x, wb.x, fmaf(xb.y, wb.y, fmaf(xb.z, wb.z, fmaf(xb.w, wb.w, a11))));
  }
  // partials [wave][row][col]; thread (r, c) sums the 4 quarters in order
  red[w * 256 + (2 * rp) * 32 + 2 * cp] = a00;
  red[w * 256 + (2 * rp) * 32 + 2 * cp + 1] = a01;
  red[w * 256 + (2 * rp + 1) * 32 + 2 * cp] = a10;
  red[w * 256 + (2 * rp + 1) * 32 + 2 * cp + 1] = a11;
  __syncthreads();
  const int r = tid >> 5, c = tid & 31;
  const int row = r0 + r, n = n0 + c;
  const float y = ((red[tid] + red[256 + tid]) + (red[512 + tid] + red[768 + tid])) +
                  (bias ? bias[n] : 0.f);
  const float ss = half_sum(row < B ? y * y : 0.f);     // this group's 32 columns
  if (row < B) {
    yws[(long long)row * N + n] = y;
    if (c == 0) ssws[(long long)cg * B + row] = ss;
  }
  if (!last_arrival(counters + rg, gridDim.x, flag)) return;
  // last block of the row group: norms (column groups in order), scaled rows;
  // every load of a thread issued before its first use
  if (row < B) {
    const int ng = gridDim.x;
    constexpr int MAXG = 32;                             // N <= 1024
    float sv[MAXG], yv[MAXG];
#pragma unroll
    for (int j = 0; j < MAXG; ++j) {
      sv[j] = j < ng ? ssws[(long long)j * B + row] : 0.f;
      yv[j] = j < ng ? yws[(long long)row * N + c + 32 * j] : 0.f;
    }
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < MAXG; ++j) s += sv[j];
    const float inv = 1.f / fmaxf(sqrtf(s), eps);
    if (c == 0) inv_norm[row] = inv;
#pragma unroll
    for (int j = 0; j < MAXG; ++j)
      if (j < ng) g[row * ldg + c + 32 * j] = yv[j] * inv;
  }
}

// dW = dy^T x [N][K] and db = colsum dy for dy [B][N] (the l2-norm backward's
// output), x [B][K].  Block = (8 rows n of dW, 64 columns k); every load of
// the block (dy [B][8], x [B][64]) in flight at once, staged in LDS; thread =
// (k, n pair): 2 x 64 FMA.  B <= 64.
constexpr int DW_N = 8, DW_K = 64;
__global__ __launch_bounds__(256) void proj_dw_kernel(
    const float* __restrict__ dy, long long lddy, const float* __restrict__ x, long long ldx,
    int B, int K, int N, float* __restrict__ dW, long long lddw, float* __restrict__ db) {
  const int tid = threadIdx.x;
  const int n0 = blockIdx.x * DW_N, k0 = blockIdx.y * DW_K;
  float* xs = (float*)g_smem;                  // [B][DW_K + 1]
  float* ds = xs + 64 * (DW_K + 1);            // [B][DW_N]
  {
    float xv[16], dv[2];
#pragma unroll
    for (int u = 0; u < 16; ++u) {             // x: 64 rows x 64 k = 16 per thread
      const int i = u * 256 + tid, b = i / DW_K, k = k0 + i % DW_K;
      xv[u] = b < B && k < K ? x[(long long)b * ldx + k] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {              // dy: 64 rows x 8 n
      const int i = u * 256 + tid, b = i / DW_N, n = n0 + i % DW_N;
      dv[u] = b < B && n < N ? dy[(long long)b * lddy + n] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int i = u * 256 + tid;
      xs[(i / DW_K) * (DW_K + 1) + i % DW_K] = xv[u];
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) ds[u * 256 + tid] = dv[u];
  }
  __syncthreads();
  const int kl = tid & 63, np = tid >> 6;      // n = n0 + np, n0 + np + 4
  float a0 = 0.f, a1 = 0.f;
  for (int b = 0; b < B; ++b) {
    const float xv = xs[b * (DW_K + 1) + kl];
    a0 = fmaf(ds[b * DW_N + np], xv, a0);
    a1 = fmaf(ds[b * DW_N + np + 4], xv, a1);
  }
  if (k0 + kl < K) {
    if (n0 + np < N) dW[(long long)(n0 + np) * lddw + k0 + kl] = a0;
    if (n0 + np + 4 < N) dW[(long long)(n0 + np + 4) * lddw + k0 + kl] = a1;
  }
  if (db && blockIdx.y == 0 && tid < DW_N && n0 + tid < N) {
    float s = 0.f;
    for (int b = 0; b < B; ++b) s += ds[b * DW_N + tid];
    db[n0 + tid] = s;
  }
}

// part[s][b][d] = sum over the chunk's classes c of dcs[b][c] W[c][d].
// Block = (class chunk s, 16 rows).  The chunk is walked in sub-chunks of
// `sub` classes (sub x D <= 24576 floats): each sub-chunk's W rows and dcs
// values are staged in LDS with every load of the block in flight at once
// (24 float4 per thread), then thread = (row half, d pair) accumulates 8 rows
// x 2 columns.  LDS: W [sub][D] | dcs transposed [sub][16].
constexpr int AD_WF = 24576;            // W floats per staged sub-chunk
__global__ __launch_bounds__(256) void arc_dx_part_kernel(
    const float* __restrict__ dcs, const float* __restrict__ W, long long ldw, int B, int C,
    int D, int chunk, int sub, float* __restrict__ part) {
  const int tid = threadIdx.x;
  const int s = blockIdx.x, r0 = blockIdx.y * AD_ROWS;
  const int cb = s * chunk, ce = min(C, cb + chunk);
  float* wl = (float*)g_smem;                   // [sub][D]
  float* dct = wl + AD_WF;                      // [sub][16]
  const int D4 = D / 4, half = tid >> 7, pl = tid & 127;
  const float* dh = dct + 8 * half;
  constexpr int NP = 3;                         // d pairs per thread (D <= 768)
  float2 acc[NP][8];
#pragma unroll
  for (int j = 0; j < NP; ++j)
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[j][i] = make_float2(0.f, 0.f);
  for (int c0 = cb; c0 < ce; c0 += sub) {
    const int nc = min(sub, ce - c0);
    if (c0 > cb) __syncthreads();               // the previous sub-chunk is consumed
    {
      constexpr int U = AD_WF / 4 / 256;
      float4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = u * 256 + tid, c = i / D4, q = i % D4;
        v[u] = c < nc ? *(const float4*)(W + (long long)(c0 + c) * ldw + 4 * q)
                      : make_float4(0.f, 0.f, 0.f, 0.f);
      }
      // dcs: nc x 16 values, at most 6 per thread (sub <= 96)
      float e[6];
#pragma unroll
      for (int u = 0; u < 6; ++u) {
        const int i = u * 256 + tid, r = i / sub, c = i % sub;
        e[u] = r < AD_ROWS && c < nc && r0 + r < B ? dcs[(long long)(r0 + r) * C + c0 + c] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = u * 256 + tid, c = i / D4, q = i % D4;
        if (c < nc) *(float4*)(wl + c * D + 4 * q) = v[u];
      }
#pragma unroll
      for (int u = 0; u < 6; ++u) {
        const int i = u * 256 + tid, r = i / sub, c = i % sub;
        if (r < AD_ROWS) dct[c * AD_ROWS + r] = e[u];
      }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < NP; ++j) {
      const int p = pl + 128 * j;
      if (2 * p >= D) break;
      for (int c = 0; c < nc; ++c) {
        const float2 wv = *(const float2*)(wl + c * D + 2 * p);
        const float4 e0 = *(const float4*)(dh + c * AD_ROWS);
        const float4 e1 = *(const float4*)(dh + c * AD_ROWS + 4);
        const float dv[8] = {e0.x, e0.y, e0.z, e0.w, e1.x, e1.y, e1.z, e1.w};
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          acc[j][i].x = fmaf(dv[i], wv.x, acc[j][i].x);
          acc[j][i].y = fmaf(dv[i], wv.y, acc[j][i].y);
        }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < NP; ++j) {
    const int p = pl + 128 * j;
    if (2 * p >= D) break;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int b = r0 + 8 * half + i;
      if (b < B) *(float2*)(part + ((long long)s * B + b) * D + 2 * p) = acc[j][i];
    }
  }
}

// dxn = sum_s part[s] (chunk order); dx = (dxn - xn (xn . dxn)) inv_nx
// (l2norm_rows_bwd_kernel's arithmetic).  Block = one row; thread = (group of
// chunks q = tid / 64, float4 column lane): a group's loads all in flight, the
// 4 groups added through LDS in order; D walked in 256-column pieces.
constexpr int AF_U = 16;                 // chunks per group (S <= 64)
__global__ __launch_bounds__(256) void arc_dx_finish_kernel(
    const float* __restrict__ part, int S, const float* __restrict__ xn,
    const float* __restrict__ inv_nx, int B, int D, float eps, float* __restrict__ dx) {
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, q = tid >> 6;
  float4* red = (float4*)g_smem;         // [4][64]
  float* row = (float*)(red + 256);      // dxn [D]
  float* dred = row + 1024;              // [4]
  float dot = 0.f;
  for (int d0 = 0; d0 < D; d0 += 256) {
    const int d = d0 + 4 * lane;
    float4 v[AF_U];
#pragma unroll
    for (int u = 0; u < AF_U; ++u) {
      const int s = q * AF_U + u;
      v[u] = s < S && d < D ? *(const float4*)(part + ((long long)s * B + b) * D + d)
                            : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int u = 0; u < AF_U; ++u) {
      a.x += v[u].x;
      a.y += v[u].y;
      a.z += v[u].z;
      a.w += v[u].w;
    }
    if (d0) __syncthreads();             // red of the previous piece consumed
    red[q * 64 + lane] = a;
    __syncthreads();
    if (q == 0 && d < D) {
      const float4 r1 = red[64 + lane], r2 = red[128 + lane], r3 = red[192 + lane];
      a = make_float4(((a.x + r1.x) + r2.x) + r3.x, ((a.y + r1.y) + r2.y) + r3.y,
                      ((a.z + r1.z) + r2.z) + r3.z, ((a.w + r1.w) + r2.w) + r3.w);
      const float4 xv = *(const float4*)(xn + (long long)b * D + d);
      dot = fmaf(xv.x, a.x, fmaf(xv.y, a.y, fmaf(xv.z, a.z, fmaf(xv.w, a.w, dot))));
      *(float4*)(row + d) = a;
    }
  }
  if (q) return;
  const float inv = inv_nx[b];
  dot = inv >= 1.f / eps ? 0.f : wave_sum(dot);
  (void)dred;
  for (int d = 4 * lane; d < D; d += 256) {
    const float4 a = *(const float4*)(row + d);
    const float4 xv = *(const float4*)(xn + (long long)b * D + d);
    *(float4*)(dx + (long long)b * D + d) =
        make_float4((a.x - xv.x * dot) * inv, (a.y - xv.y * dot) * inv,
                    (a.z - xv.z * dot) * inv, (a.w - xv.w * dot) * inv);
  }
}

// class chunks of the dxn partials: ~96 classes each, at most 64 (the finish
// kernel's 4 groups of AF_U)
int arc_dx_chunks(int B, int C) {
  (void)B;
  return std::max(1, std::min(64, (C + 95) / 96));
}

bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

}  // namespace

extern "C" {

int tgfr_proj_l2norm_ws(int B, int N, long long* floats) {
  if (B <= 0 || N <= 0 || !floats) return 1001;
  *floats = (long long)B * N + (long long)(N / PJ_COLS) * B;
  return 0;
}

int tgfr_proj_l2norm_fwd(const float* x, long long ldx, int B, int K, const float* W,
                         long long ldw, const float* bias, int N, float eps, float* ws,
                         float* g, long long ldg, float* inv_norm, unsigned* counters,
                         void* stream) {
  if (B <= 0 || K <= 0 || N <= 0 || K % 4 || N % PJ_COLS || N > 1024 ||
      (PJ_COLS + PJ_ROWS) * (K / 4) > PJ_STG * 256 || (ldx & 3) ||
      (ldw & 3) || !al16(x) || !al16(W) || !ws || !counters)
    return 1001;
  const int lds = ((PJ_COLS + PJ_ROWS) * (K + 4) + 4 * 256) * 4 + 16;
  if (lds > 65536) {
    static bool once = [] {
      return hipFuncSetAttribute((const void*)proj_fwd_kernel,
                                 hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) ==
             hipSuccess;
    }();
    if (!once) return 1003;
  }
  const dim3 grid(N / PJ_COLS, (B + PJ_ROWS - 1) / PJ_ROWS);
  hipLaunchKernelGGL(proj_fwd_kernel, grid, dim3(256), lds, (hipStream_t)stream, x, ldx, B, K,
                     W, ldw, bias, N, eps, ws, ws + (long long)B * N, g, ldg, inv_norm, counters);
  return (int)hipGetLastError();
}

int tgfr_proj_dw(const float* dy, long long lddy, const float* x, long long ldx, int B, int K,
                 int N, float* dW, long long lddw, float* db, void* stream) {
  if (B <= 0 || B > 64 || K <= 0 || N <= 0 || !dy || !x || !dW) return 1001;
  hipLaunchKernelGGL(proj_dw_kernel, dim3((N + DW_N - 1) / DW_N, (K + DW_K - 1) / DW_K),
                     dim3(256), (64 * (DW_K + 1) + 64 * DW_N) * 4, (hipStream_t)stream, dy, lddy,
                     x, ldx, B, K, N, dW, lddw, db);
  return (int)hipGetLastError();
}

int tgfr_arc_dx_ws(int B, int C, int D, long long* floats) {
  if (B <= 0 || C <= 0 || D <= 0 || !floats) return 1001;
  *floats = (long long)arc_dx_chunks(B, C) * B * D;
  return 0;
}

int tgfr_arc_dx(const float* dcs, const float* W, long long ldw, int B, int C, int D,
                const float* xn, const float* inv_nx, float eps, float* ws, float* dx,
                void* stream) {
  if (B <= 0 || C <= 0 || D <= 0 || D % 4 || D > 768 || (ldw & 3) || !al16(W) || !al16(xn) ||
      !al16(dx) || !al16(ws))
    return 1001;
  const int S = arc_dx_chunks(B, C);
  const int chunk = (C + S - 1) / S;
  const int sub = std::min(96, AD_WF / D);
  auto* s = (hipStream_t)stream;
  const int lds = (AD_WF + 96 * AD_ROWS) * 4;
  static const bool ok = hipFuncSetAttribute((const void*)arc_dx_part_kernel,
                                             hipFuncAttributeMaxDynamicSharedMemorySize,
                                             160 * 1024) == hipSuccess;
  if (!ok) return 1003;
  hipLaunchKernelGGL(arc_dx_part_kernel, dim3(S, (B + AD_ROWS - 1) / AD_ROWS), dim3(256), lds,
                     s, dcs, W, ldw, B, C, D, chunk, sub, ws);
  hipLaunchKernelGGL(arc_dx_finish_kernel, dim3(B), dim3(256), (256 * 4 + 1024 + 4) * 4, s, ws,
                     S, xn, inv_nx, B, D, eps, dx);
  return (int)hipGetLastError();
}

}  // extern "C"
