// pp3_policy.hip -- on-device MLP policy in the reference's deployment format
// (export.py:13-81 convert_params: dense layers, observation normalisation folded into the
// first layer, final layer = the mean half of the Gaussian head, final activation tanh).
//
// One workgroup = 8 waves (2 per SIMD) = a tile of 16 environments; every layer is a
// [16 x K] x [K x M] product on the f32-input matrix cores (v_mfma_f32_16x16x4_f32: exact f32
// products, f32 accumulation), the eight waves splitting the layer's 16-column output tiles.
// Activations stay in LDS between layers; weights are read straight from global memory (the
// whole MLP is a few hundred KB and stays L2-resident across workgroups) in MFMA-fragment
// order: the host stores, per 16-column tile and group of 4 k-blocks, the 64 lanes' B values
// as one float4 per lane, so one 16-byte load per lane (1 KB contiguous per wave) feeds four
// MFMAs -- a row-major layout would make every MFMA's B operand a 4-row gather.  32 k-blocks
// of a tile are in flight before its MFMAs.  A: lane l holds X[row l&15][k0 + (l>>4)],
// B: W[k0 + (l>>4)][c0 + (l&15)], C/D: col l&15, row 4(l>>4)+r.
#include <hip/hip_runtime.h>

#include <math.h>

#include <string>
#include <vector>

#include "pupper_hip.h"

namespace pp3pol {

constexpr int TILE = 16;                 // environments per workgroup
constexpr int NWAVE = 8;
constexpr int MAXW = PP3_POLICY_MAX_WIDTH;  // widest layer (padded)

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
constexpr int CG = 8;  // groups of 4 k-blocks (32 k-blocks = 128 inputs) per chunk

__global__ __launch_bounds__(64 * NWAVE) void mlp_kernel(Net net, const float* __restrict__ obs, int obs_stride,
                                                         float* __restrict__ act, int act_stride, int n) {
  __shared__ float buf[2][TILE][MAXW + 4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int row0 = blockIdx.x * TILE;
  // observation tile -> LDS (rows past n are zero)
  for (int i = tid; i < TILE * net.layer[0].Kp; i += 64 * NWAVE) {
    const int r = i / net.layer[0].Kp, k = i - r * net.layer[0].Kp;
    const int row = row0 + r;
    buf[0][r][k] = (row < n && k < net.in_dim) ? obs[(size_t)row * obs_stride + k] : 0.0f;
  }
  __syncthreads();
  int cur = 0;
  for (int li = 0; li < net.n_layers; li++) {
    const Layer L = net.layer[li];
    const float(*X)[MAXW + 4] = buf[cur];
    float(*Y)[MAXW + 4] = buf[cur ^ 1];
    const int ntile = L.Mp / TILE;
    const bool last = li == net.n_layers - 1;
    for (int t = wave; t < ntile; t += NWAVE) {
      const int c0 = t * TILE;
      // two independent accumulators (even / odd k blocks) cover the dependent MFMA latency
      f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f}, acc1 = {0.0f, 0.0f, 0.0f, 0.0f};
      const int ar = lane & 15, kk = lane >> 4;
      const int nblk = L.Kp / 4;
      for (int g0 = 0; g0 < L.ngrp; g0 += CG) {
        f32x4 bq[CG];
        float av[CG][4];
        const f32x4* wf = reinterpret_cast<const f32x4*>(L.w) + ((size_t)t * L.ngrp + g0) * 64 + lane;
#pragma unroll
        for (int q = 0; q < CG; q++) {  // every load of the chunk in flight together
          bq[q] = (g0 + q < L.ngrp) ? wf[(size_t)q * 64] : f32x4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
          for (int j = 0; j < 4; j++) {
            const int kb = 4 * (g0 + q) + j;
            av[q][j] = kb < nblk ? X[ar][4 * kb + kk] : 0.0f;
          }
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
    cur ^= 1;
  }
}

}  // namespace pp3pol

using namespace pp3pol;

struct pp3_policy {
  int device;
  Net net;
  float* dev;  // all layer weights
};

static thread_local std::string g_perr;
static int perr(int code, const std::string& m) {
  g_perr = m;
  return code;
}
#define PHIP(x)                                                                                  \
  do {                                                                                           \
    hipError_t e_ = (x);                                                                         \
    if (e_ != hipSuccess) return perr(PP3_ERR_HIP, std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

extern "C" {

const char* pp3_policy_last_error(void) { return g_perr.c_str(); }

int pp3_policy_create(int32_t device, int32_t in_dim, int32_t n_layers, const int32_t* out_dims, const int32_t* acts,
                      const float* weights, pp3_policy_t** out) {
  if (!out_dims || !acts || !weights || !out) return perr(PP3_ERR_ARG, "pp3_policy_create: null argument");
  if (n_layers < 1 || n_layers > PP3_POLICY_MAX_LAYERS) return perr(PP3_ERR_ARG, "pp3_policy_create: 1..8 layers");
  if (in_dim < 1 || in_dim > PP3_POLICY_MAX_WIDTH) return perr(PP3_ERR_ARG, "pp3_policy_create: input width");
  Net net{};
  net.n_layers = n_layers;
  net.in_dim = in_dim;
  std::vector<float> host;
  std::vector<size_t> woff(n_layers), boff(n_layers);
  int K = in_dim;
  size_t src = 0;
  for (int i = 0; i < n_layers; i++) {
    const int M = out_dims[i];
    if (M < 1 || M > PP3_POLICY_MAX_WIDTH) return perr(PP3_ERR_ARG, "pp3_policy_create: layer width 1..576");
    if (acts[i] < PP3_ACT_LINEAR || acts[i] > PP3_ACT_SIGMOID) return perr(PP3_ERR_ARG, "pp3_policy_create: activation");
    const int Kp = (K + 3) / 4 * 4, Mp = (M + TILE - 1) / TILE * TILE;
    const int ngrp = (Kp / 4 + 3) / 4, ntile = Mp / TILE;
    woff[i] = host.size();
    host.resize(host.size() + (size_t)ntile * ngrp * 256, 0.0f);
    for (int t = 0; t < ntile; t++)  // fragment order: [tile][group][lane][j] = W[4(4g+j) + lane/16][16t + lane%16]
      for (int g = 0; g < ngrp; g++)
        for (int ln = 0; ln < 64; ln++)
          for (int j = 0; j < 4; j++) {
            const int k = 4 * (4 * g + j) + (ln >> 4), m = TILE * t + (ln & 15);
            if (k < K && m < M)
              host[woff[i] + (((size_t)t * ngrp + g) * 64 + ln) * 4 + j] = weights[src + (size_t)k * M + m];
          }
    src += (size_t)K * M;
    boff[i] = host.size();
    host.resize(host.size() + Mp, 0.0f);
    for (int m = 0; m < M; m++) host[boff[i] + m] = weights[src + m];
    src += M;
    net.layer[i].K = K; net.layer[i].Kp = Kp; net.layer[i].M = M; net.layer[i].Mp = Mp; net.layer[i].act = acts[i];
    net.layer[i].ngrp = ngrp;
    K = M;
  }
  net.out_dim = K;
  pp3_policy* p = new pp3_policy();
  p->device = device;
  if (hipSetDevice(device) != hipSuccess || hipMalloc(&p->dev, host.size() * sizeof(float)) != hipSuccess) {
    delete p;
    return perr(PP3_ERR_HIP, "pp3_policy_create: device allocation failed");
  }
  PHIP(hipMemcpy(p->dev, host.data(), host.size() * sizeof(float), hipMemcpyHostToDevice));
  for (int i = 0; i < n_layers; i++) {
    net.layer[i].w = p->dev + woff[i];
    net.layer[i].b = p->dev + boff[i];
  }
  p->net = net;
  *out = p;
  return PP3_OK;
}

int pp3_policy_act(pp3_policy_t* p, const float* obs_dev, int64_t obs_stride, int32_t n, float* actions_dev,
                   int64_t action_stride, void* stream) {
  if (!p || !obs_dev || !actions_dev) return perr(PP3_ERR_ARG, "pp3_policy_act: null argument");
  if (n <= 0) return PP3_OK;
  if (obs_stride < p->net.in_dim) return perr(PP3_ERR_ARG, "pp3_policy_act: observation row shorter than in_dim");
  if (action_stride < p->net.out_dim) return perr(PP3_ERR_ARG, "pp3_policy_act: action row shorter than out_dim");
  PHIP(hipSetDevice(p->device));
  hipLaunchKernelGGL(mlp_kernel, dim3((n + TILE - 1) / TILE), dim3(64 * NWAVE), 0, (hipStream_t)stream, p->net,
                     obs_dev, (int)obs_stride, actions_dev, (int)action_stride, n);
  PHIP(hipGetLastError());
  return PP3_OK;
}

int pp3_policy_out_dim(const pp3_policy_t* p) { return p ? p->net.out_dim : 0; }

int pp3_policy_destroy(pp3_policy_t* p) {
  if (!p) return PP3_OK;
  (void)hipSetDevice(p->device);
  (void)hipFree(p->dev);
  delete p;
  return PP3_OK;
}

}  // extern "C"
