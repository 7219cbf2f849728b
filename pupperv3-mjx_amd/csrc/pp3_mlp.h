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
constexpr int CG = 8;                       // groups of 4 k-blocks (32 k-blocks = 128 inputs) per chunk

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
__device__ __forceinline__ void load_chunk(const Layer& L, int t, int g0, int lane, f32x4 (&bq)[CG]) {
  const f32x4* wf = reinterpret_cast<const f32x4*>(L.w) + ((size_t)t * L.ngrp + g0) * 64 + lane;
#pragma unroll
  for (int q = 0; q < CG; q++) bq[q] = (g0 + q < L.ngrp) ? wf[(size_t)q * 64] : f32x4{0.0f, 0.0f, 0.0f, 0.0f};
}

template <class NetT>
__device__ __forceinline__ Layer layer_of(NetT& net, int li) {
  Layer L;  // (field by field: a constant-address-space record has no copy constructor)
  L.w = net.layer[li].w; L.b = net.layer[li].b; L.K = net.layer[li].K; L.Kp = net.layer[li].Kp;
  L.M = net.layer[li].M; L.Mp = net.layer[li].Mp; L.act = net.layer[li].act; L.ngrp = net.layer[li].ngrp;
  return L;
}

// The MLP of observation rows row0 .. row0+15 (rows >= n read as zero, get no action) ->
// act[row * act_stride + col] for col < out_dim.  Called by all 64 * NWAVE threads of the
// workgroup (tid = threadIdx.x); `buf` is the workgroup's LDS scratch.  Ends with a barrier.
// NetT: Net (a kernel's by-value argument) or KNet.  PF (the fused rollout, which has the
// registers): every weight chunk's loads are issued one chunk ahead -- the next chunk of the
// tile, else the next tile's first, else the first chunk of this wave's first tile in the next
// layer, across the epilogue and barrier -- and the very first before the observation tile is
// staged.  Only the issue points of loads move: the MFMA sequence, and so the result, is the
// same with and without.  `in` (InT = float[TILE][W] in LDS, W >= in_dim, in_dim a multiple of
// 4): the observation rows are already there (written by the env step, a barrier since), so the
// first layer reads them in place instead of staging `obs` from global memory; rows past n may
// hold anything (a row's outputs depend on that row only, and they are not stored).
template <class NetT, bool PF = false, class BufT = TileBuf, class InT = TileRows>
__device__ __forceinline__ void mlp_tile(NetT& net, const float* __restrict__ obs, int obs_stride,
                                         float* __restrict__ act, int act_stride, int n, int row0, BufT& buf,
                                         int tid, InT* in = nullptr) {
  const int lane = tid & 63, wave = tid >> 6;
  f32x4 nxt[CG];  // PF: the next chunk's B fragments, in flight
  if (PF) {
    const Layer L0 = layer_of(net, 0);
    if (wave < L0.Mp / TILE) load_chunk(L0, wave, 0, lane, nxt);
  }
  if (!in) {
    // observation tile -> LDS (rows past n are zero)
    for (int i = tid; i < TILE * net.layer[0].Kp; i += 64 * NWAVE) {
      const int r = i / net.layer[0].Kp, k = i - r * net.layer[0].Kp;
      const int row = row0 + r;
      buf[0][r][k] = (row < n && k < net.in_dim) ? obs[(size_t)row * obs_stride + k] : 0.0f;
    }
    __syncthreads();
  }
  // one layer's output tiles of this wave: X the [TILE][.] input rows, Y the output rows
  auto layer = [&](auto& X, auto& Y, const Layer& L, int li, bool last) {
    const int ntile = L.Mp / TILE;
    for (int t = wave; t < ntile; t += NWAVE) {
      const int c0 = t * TILE;
      // two independent accumulators (even / odd k blocks) cover the dependent MFMA latency
      f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f}, acc1 = {0.0f, 0.0f, 0.0f, 0.0f};
      const int ar = lane & 15, kk = lane >> 4;
      const int nblk = L.Kp / 4;
      for (int g0 = 0; g0 < L.ngrp; g0 += CG) {
        f32x4 bq[CG];
        float av[CG][4];
        if (PF) {
#pragma unroll
          for (int q = 0; q < CG; q++) bq[q] = nxt[q];
          // the next chunk: this tile's, the next tile's of this layer, or the next layer's first
          if (g0 + CG < L.ngrp) {
            load_chunk(L, t, g0 + CG, lane, nxt);
          } else if (t + NWAVE < ntile) {
            load_chunk(L, t + NWAVE, 0, lane, nxt);
          } else if (!last) {
            const Layer Ln = layer_of(net, li + 1);
            if (wave < Ln.Mp / TILE) load_chunk(Ln, wave, 0, lane, nxt);
          }
        } else {
          load_chunk(L, t, g0, lane, bq);  // every load of the chunk in flight together
        }
#pragma unroll
        for (int q = 0; q < CG; q++)
#pragma unroll
          for (int j = 0; j < 4; j++) {
            const int kb = 4 * (g0 + q) + j;
            av[q][j] = kb < nblk ? X[ar][4 * kb + kk] : 0.0f;
          }
#pragma unroll
        for (int q = 0; q < CG; q++) {
          if (g0 + q < L.ngrp) {  // uniform; padded blocks of a ragged group multiply zeros
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[q][0], bq[q].x, acc, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av[q][1], bq[q].y, acc1, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[q][2], bq[q].z, acc, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av[q][3], bq[q].w, acc1, 0, 0, 0);
          }
        }
      }
      acc += acc1;
      const int col = c0 + (lane & 15);
      const float bias = L.b[col];
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
  for (int li = 0; li < net.n_layers; li++) {
    const Layer L = layer_of(net, li);
    const bool last = li == net.n_layers - 1;
    if (li == 0 && in) layer(*in, buf[1], L, li, last);
    else layer(buf[cur], buf[cur ^ 1], L, li, last);
    cur ^= 1;
  }
}

}  // namespace pp3pol

// the device-side network of a policy handle (pp3_policy.hip; C++ linkage, not part of the C ABI)
const pp3pol::Net* pp3_policy_net(const pp3_policy_t* p);
int pp3_policy_device(const pp3_policy_t* p);
