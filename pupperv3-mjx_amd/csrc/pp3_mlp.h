// pp3_mlp.h -- the exported-format policy MLP on one 16-environment tile, shared by the
// stand-alone policy kernel (pp3_policy.hip mlp_kernel: pp3_policy_act) and the fused
// policy-in-the-loop rollout (pp3_env.hip env_step_kernel<NC, true, 8>: pp3_rollout_policy).
// One source for both, so the two compute the same instructions and give bit-identical actions.
//
// Format: export.py:13-81 convert_params (dense layers, observation normalisation folded into
// the first layer, final layer = the mean half of the Gaussian head, final activation tanh).
// Every layer is a [16 x K] x [K x M] product on the f32-input matrix cores
// (v_mfma_f32_16x16x4_f32: exact f32 products, f32 accumulation), the eight waves splitting the
// layer's 16-column output tiles.  Activations stay in LDS between layers; weights are read
// straight from global memory (the whole MLP is a few hundred KB and stays L2-resident) in
// MFMA-fragment order: the host stores, per 16-column tile and group of 4 k-blocks, the 64 lanes'
// B values as one float4 per lane, so one 16-byte load per lane (1 KB contiguous per wave) feeds
// four MFMAs.  32 k-blocks of a tile are in flight before its MFMAs.  A: lane l holds
// X[row l&15][k0 + (l>>4)], B: W[k0 + (l>>4)][c0 + (l&15)], C/D: col l&15, row 4(l>>4)+r.
#pragma once

#include <hip/hip_runtime.h>

#include <math.h>

#include "pupper_hip.h"

namespace pp3pol {

constexpr int TILE = 16;                    // environments per tile (one workgroup)
constexpr int NWAVE = 8;                    // waves per tile
constexpr int MAXW = PP3_POLICY_MAX_WIDTH;  // widest layer (padded)
constexpr int CG8 = 8;                      // groups of 4 k-blocks (32 k-blocks = 128 inputs) per chunk

struct Layer {
  const float* w;  // fragment order [Mp/16][ngrp][64 lanes][4], zero padded
  const float* b;  // [Mp]
  int K, Kp, M, Mp, act;
  int ngrp;  // groups of 4 k-blocks (16 inputs)
};
struct Net {
  Layer layer[PP3_POLICY_MAX_LAYERS];
  int n_layers, in_dim, out_dim;
};

// LDS activations of one tile: two buffers of [TILE][MAXW + 4] floats (74 KB)
typedef float TileBuf[2][TILE][MAXW + 4];
typedef float TileRows[TILE][MAXW + 4];  // one of the two
typedef __attribute__((address_space(3))) float LdsTileBuf[2][TILE][MAXW + 4];  // (explicitly LDS)
constexpr size_t TILE_BUF_BYTES = sizeof(TileBuf);

__device__ __forceinline__ float activate(float x, int act) {
  switch (act) {
    case PP3_ACT_RELU: return fmaxf(x, 0.0f);
    case PP3_ACT_ELU: return x > 0.0f ? x : expm1f(x);
    case PP3_ACT_TANH: return tanhf(x);
    case PP3_ACT_SIGMOID: return 1.0f / (1.0f + expf(-x));
    default: return x;
  }
}

typedef float f32x4 __attribute__((ext_vector_type(4)));

// The network as the fused rollout sees it: inside its kernel arguments (constant address space,
// so the layer records are scalar loads)
typedef __attribute__((address_space(4))) const Net KNet;

// One chunk (CG groups of 4 k-blocks) of tile t's B fragments, starting at group g0 (groups past
// ngrp read as zero)
template <int CG>
__device__ __forceinline__ void load_chunk(const Layer& L, int t, int g0, int lane, f32x4 (&bq)[CG]) {
  const f32x4* wf = reinterpret_cast<const f32x4*>(L.w) + ((size_t)t * L.ngrp + g0) * 64 + lane;
#pragma unroll
  for (int q = 0; q < CG; q++) bq[q] = (g0 + q < L.ngrp) ? wf[(size_t)q * 64] : f32x4{0.0f, 0.0f, 0.0f, 0.0f};
}

// wave-uniform values kept in SGPRs: an out-of-line caller passes them in VGPRs (the function ABI),
// which would make every loop bound and predicate below look divergent (exec-mask branches
// around each load); readfirstlane of a value already in an SGPR is free
__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
template <class T>
__device__ __forceinline__ T* uni(T* p) {
  const uint64_t v = (uint64_t)(uintptr_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v), hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return (T*)(uintptr_t)(((uint64_t)hi << 32) | lo);
}

// the same for a chunk that lies wholly inside the layer (no predicates)
template <int CG>
__device__ __forceinline__ void load_chunk_full(const Layer& L, int t, int g0, int lane, f32x4 (&bq)[CG]) {
  const f32x4* wf = reinterpret_cast<const f32x4*>(L.w) + ((size_t)t * L.ngrp + g0) * 64 + lane;
#pragma unroll
  for (int q = 0; q < CG; q++) bq[q] = wf[(size_t)q * 64];
}

template <class NetT>
__device__ __forceinline__ Layer layer_of(NetT& net, int li) {
  Layer L;  // (field by field: a constant-address-space record has no copy constructor)
  L.w = uni(net.layer[li].w); L.b = uni(net.layer[li].b); L.K = uni(net.layer[li].K); L.Kp = uni(net.layer[li].Kp);
  L.M = uni(net.layer[li].M); L.Mp = uni(net.layer[li].Mp); L.act = uni(net.layer[li].act);
  L.ngrp = uni(net.layer[li].ngrp);
  return L;
}

// The MLP of observation rows row0 .. row0+15 (rows >= n read as zero, get no action) ->
// act[row * act_stride + col] for col < out_dim.  Called by all 64 * NWAVE threads of the
// workgroup (tid = threadIdx.x); `buf` is the workgroup's LDS scratch.  Ends with a barrier.
// NetT: Net (a kernel's by-value argument) or KNet.  Weight chunks are loaded where they are
// multiplied (a one-chunk-ahead prefetch measured slower: profiles/AB_LOG.md).  `in` (InT = float[TILE][W] in LDS, W >= in_dim, in_dim a multiple of
// 4): the observation rows are already there (written by the env step, a barrier since), so the
// first layer reads them in place instead of staging `obs` from global memory; rows past n may
// hold anything (a row's outputs depend on that row only, and they are not stored).
// CG: groups of 4 k-blocks per chunk (8 in the stand-alone kernel; the fused rollout's out-of-line
// call uses 4, whose registers fit the callee's caller-saved VGPRs: no save / restore through
// scratch per call).  The MFMA sequence does not depend on it.
template <class NetT, class BufT = TileBuf, class InT = TileRows, int CG = CG8>
__device__ __forceinline__ void mlp_tile(NetT& net, const float* __restrict__ obs, int obs_stride,
                                         float* __restrict__ act, int act_stride, int n, int row0, BufT& buf,
                                         int tid, InT* in = nullptr) {
  // the wave index is wave-uniform: readfirstlane says so, so the tile / chunk / group loops below
  // become scalar branches instead of exec-mask divergence
  const int lane = tid & 63, wave = uni(tid >> 6);
  n = uni(n);
  row0 = uni(row0);
  act = uni(act);
  act_stride = uni(act_stride);
  if (!in) {
    // observation tile -> LDS (rows past n are zero)
    const int kp0 = uni(net.layer[0].Kp), in_dim = uni(net.in_dim);
    obs = uni(obs);
    obs_stride = uni(obs_stride);
    for (int i = tid; i < TILE * kp0; i += 64 * NWAVE) {
      const int r = i / kp0, k = i - r * kp0;
      const int row = row0 + r;
      buf[0][r][k] = (row < n && k < in_dim) ? obs[(size_t)row * obs_stride + k] : 0.0f;
    }
    __syncthreads();
  }
  // one layer's output tiles of this wave: X the [TILE][.] input rows, Y the output rows
  auto layer = [&](auto& X, auto& Y, const Layer& L, bool last) {
    const int ntile = L.Mp / TILE;
    for (int t = wave; t < ntile; t += NWAVE) {
      const int c0 = t * TILE;
      const int col = c0 + (lane & 15);
      const float bias = L.b[col];  // (issued before the weight chunks: its wait never waits for them)
      // two independent accumulators (even / odd k blocks) cover the dependent MFMA latency
      f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f}, acc1 = {0.0f, 0.0f, 0.0f, 0.0f};
      const int ar = lane & 15, kk = lane >> 4;
      const int nblk = L.Kp / 4;
      for (int g0 = 0; g0 < L.ngrp; g0 += CG) {
        // a whole chunk (every group and k block inside the layer) runs without per-element
        // predicates; the ragged last chunk keeps them.  The MFMA sequence is the same either way.
        const bool full = g0 + CG <= L.ngrp && 4 * (g0 + CG) <= nblk;
        f32x4 bq[CG];
        float av[CG][4];
        if (full) {
          load_chunk_full(L, t, g0, lane, bq);
        } else {
          load_chunk(L, t, g0, lane, bq);  // every load of the chunk in flight together
        }
        if (full) {
#pragma unroll
          for (int q = 0; q < CG; q++)
#pragma unroll
            for (int j = 0; j < 4; j++) av[q][j] = X[ar][4 * (4 * (g0 + q) + j) + kk];
        } else {
#pragma unroll
          for (int q = 0; q < CG; q++)
#pragma unroll
            for (int j = 0; j < 4; j++) {
              const int kb = 4 * (g0 + q) + j;
              av[q][j] = kb < nblk ? X[ar][4 * kb + kk] : 0.0f;
            }
        }
#pragma unroll
        for (int q = 0; q < CG; q++) {
          if (full || g0 + q < L.ngrp) {  // uniform; padded blocks of a ragged group multiply zeros
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[q][0], bq[q].x, acc, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av[q][1], bq[q].y, acc1, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[q][2], bq[q].z, acc, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av[q][3], bq[q].w, acc1, 0, 0, 0);
          }
        }
      }
      acc += acc1;
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const int row = 4 * (lane >> 4) + r;
        const float v = activate(acc[r] + bias, L.act);
        if (!last) {
          Y[row][col] = v;
        } else if (col < L.M && row0 + row < n) {
          act[(size_t)(row0 + row) * act_stride + col] = v;
        }
      }
    }
    __syncthreads();
  };
  int cur = 0;
  const int n_layers = uni(net.n_layers);
  for (int li = 0; li < n_layers; li++) {
    const Layer L = layer_of(net, li);
    const bool last = li == n_layers - 1;
    if (li == 0 && in) layer(*in, buf[1], L, last);
    else layer(buf[cur], buf[cur ^ 1], L, last);
    cur ^= 1;
  }
}

}  // namespace pp3pol

// the device-side network of a policy handle (pp3_policy.hip; C++ linkage, not part of the C ABI)
const pp3pol::Net* pp3_policy_net(const pp3_policy_t* p);
int pp3_policy_device(const pp3_policy_t* p);
