// pp3_policy.hip -- on-device MLP policy in the reference's deployment format
// (export.py:13-81 convert_params: dense layers, observation normalisation folded into the
// first layer, final layer = the mean half of the Gaussian head, final activation tanh).
//
// One workgroup = 8 waves (2 per SIMD) = a tile of 16 environments; the tile's MLP is
// pp3_mlp.h mlp_tile (f32 MFMA layer products, activations in LDS, weights in MFMA-fragment
// order), the same code the fused policy rollout runs inside the env step kernel.
#include <hip/hip_runtime.h>

#include <math.h>

#include <string>
#include <vector>

#include "pp3_mlp.h"
#include "pupper_hip.h"

namespace pp3pol {

__global__ __launch_bounds__(64 * NWAVE) void mlp_kernel(Net net, const float* __restrict__ obs, int obs_stride,
                                                         float* __restrict__ act, int act_stride, int n) {
  __shared__ TileBuf buf;
  mlp_tile(net, obs, obs_stride, act, act_stride, n, blockIdx.x * TILE, buf, threadIdx.x);
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

}  // extern "C"

const pp3pol::Net* pp3_policy_net(const pp3_policy_t* p) { return p ? &p->net : nullptr; }
int pp3_policy_device(const pp3_policy_t* p) { return p ? p->device : -1; }

extern "C" {

int pp3_policy_destroy(pp3_policy_t* p) {
  if (!p) return PP3_OK;
  (void)hipSetDevice(p->device);
  (void)hipFree(p->dev);
  delete p;
  return PP3_OK;
}

}  // extern "C"
