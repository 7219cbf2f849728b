// pp3_render.hip -- batched z-buffer rasteriser behind PupperV3Env.render (environment.py:545-547,
// Brax PipelineEnv.render -> MuJoCo's renderer; used for the policy videos of utils.py:214-293).
//
// Not on the training path.  The host (pupperv3_mjx/render.py) turns the model's visual geoms
// into one triangle soup in geom-local frames (STL meshes when the mesh files are present, else
// primitive proxies), and per frame the world transform of every geom and the camera basis.  Two
// launches per batch of frames:
//   raster_kernel:  one thread per (triangle, frame): transform, project (pinhole, MuJoCo's fovy),
//                   headlight Lambert shade, walk the pixel centres of its clipped bounding box,
//                   and keep the nearest fragment per pixel with a 64-bit atomicMin of
//                   (camera depth bits << 32 | rgb) -- order-independent, so the image is
//                   deterministic whatever the thread order;
//   resolve_kernel: one thread per pixel: the fragment, or the floor plane (builtin checker of
//                   the grid material, texuniform: squares of `check` metres), or the gradient
//                   skybox, written as u8 RGB.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <string>

#include "pupper_hip.h"

namespace pp3r {

constexpr float NEAR = 1e-3f;
constexpr unsigned long long EMPTY = ~0ull;

// camera record: pos[3], right[3], up[3], fwd[3], f_px (pixels), 3 pad
struct Cam {
  float pos[3], right[3], up[3], fwd[3], fpx, pad[3];
};
static_assert(sizeof(Cam) == 16 * sizeof(float), "Cam layout");

__device__ __forceinline__ float edgef(float ax, float ay, float bx, float by, float px, float py) {
  return (bx - ax) * (py - ay) - (by - ay) * (px - ax);
}

__global__ void raster_kernel(const float* __restrict__ tris, const int32_t* __restrict__ tri_geom, int ntri,
                              const float* __restrict__ geom_rgb, const float* __restrict__ xf, int ngeom,
                              const Cam* __restrict__ cams, int H, int W, float ambient, float diffuse,
                              unsigned long long* __restrict__ zbuf) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  const int f = blockIdx.y;
  if (t >= ntri) return;
  const int g = tri_geom[t];
  const float* X = xf + ((size_t)f * ngeom + g) * 12;  // R (row-major 3x3), then translation
  const Cam c = cams[f];
  float w[3][3], cc[3][3];
#pragma unroll
  for (int k = 0; k < 3; k++) {
    const float* v = tris + (size_t)t * 9 + 3 * k;
#pragma unroll
    for (int i = 0; i < 3; i++) w[k][i] = X[3 * i] * v[0] + X[3 * i + 1] * v[1] + X[3 * i + 2] * v[2] + X[9 + i];
    const float r0 = w[k][0] - c.pos[0], r1 = w[k][1] - c.pos[1], r2 = w[k][2] - c.pos[2];
    cc[k][0] = r0 * c.right[0] + r1 * c.right[1] + r2 * c.right[2];
    cc[k][1] = r0 * c.up[0] + r1 * c.up[1] + r2 * c.up[2];
    cc[k][2] = r0 * c.fwd[0] + r1 * c.fwd[1] + r2 * c.fwd[2];
    if (cc[k][2] < NEAR) return;  // (no near-plane clipping: the tracking camera never cuts the scene)
  }
  // headlight Lambert shading on the face normal, two-sided
  const float e1[3] = {w[1][0] - w[0][0], w[1][1] - w[0][1], w[1][2] - w[0][2]};
  const float e2[3] = {w[2][0] - w[0][0], w[2][1] - w[0][1], w[2][2] - w[0][2]};
  const float n[3] = {e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2], e1[0] * e2[1] - e1[1] * e2[0]};
  const float nn = sqrtf(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
  if (nn <= 0.0f) return;
  const float lam = fabsf(n[0] * c.fwd[0] + n[1] * c.fwd[1] + n[2] * c.fwd[2]) / nn;
  const float sh = fminf(ambient + diffuse * lam, 1.0f);
  uint32_t rgb = 0;
#pragma unroll
  for (int i = 0; i < 3; i++) {
    const float v = fminf(fmaxf(geom_rgb[3 * g + i] * sh, 0.0f), 1.0f);
    rgb |= (uint32_t)(v * 255.0f + 0.5f) << (8 * i);
  }
  float sx[3], sy[3];
#pragma unroll
  for (int k = 0; k < 3; k++) {
    sx[k] = 0.5f * W + c.fpx * cc[k][0] / cc[k][2];
    sy[k] = 0.5f * H - c.fpx * cc[k][1] / cc[k][2];
  }
  const float area = edgef(sx[0], sy[0], sx[1], sy[1], sx[2], sy[2]);
  if (fabsf(area) < 1e-12f) return;
  const float ia = 1.0f / area;
  const int x0 = max(0, (int)floorf(fminf(sx[0], fminf(sx[1], sx[2])))), x1 = min(W - 1, (int)ceilf(fmaxf(sx[0], fmaxf(sx[1], sx[2]))));
  const int y0 = max(0, (int)floorf(fminf(sy[0], fminf(sy[1], sy[2])))), y1 = min(H - 1, (int)ceilf(fmaxf(sy[0], fmaxf(sy[1], sy[2]))));
  const float iz0 = 1.0f / cc[0][2], iz1 = 1.0f / cc[1][2], iz2 = 1.0f / cc[2][2];
  unsigned long long* zb = zbuf + (size_t)f * H * W;
  for (int py = y0; py <= y1; py++) {
    const float fy = py + 0.5f;
    for (int px = x0; px <= x1; px++) {
      const float fx = px + 0.5f;
      const float b0 = edgef(sx[1], sy[1], sx[2], sy[2], fx, fy) * ia;
      const float b1 = edgef(sx[2], sy[2], sx[0], sy[0], fx, fy) * ia;
      const float b2 = edgef(sx[0], sy[0], sx[1], sy[1], fx, fy) * ia;
      if (b0 < 0.0f || b1 < 0.0f || b2 < 0.0f) continue;
      const float depth = 1.0f / (b0 * iz0 + b1 * iz1 + b2 * iz2);  // perspective-correct camera depth
      const unsigned long long key = ((unsigned long long)__float_as_uint(depth) << 32) | rgb;
      atomicMin(zb + (size_t)py * W + px, key);
    }
  }
}

struct Env {
  float floor_rgb1[3], floor_rgb2[3], check, floor_z;
  float sky_top[3], sky_bottom[3];
  float ambient, diffuse;
  int floor_on, pad;
};

__global__ void resolve_kernel(const unsigned long long* __restrict__ zbuf, const Cam* __restrict__ cams, int F, int H,
                               int W, Env env, uint8_t* __restrict__ out) {
  const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (size_t)F * H * W) return;
  const int f = (int)(idx / ((size_t)H * W));
  const int rem = (int)(idx - (size_t)f * H * W);
  const int py = rem / W, px = rem - py * W;
  const Cam c = cams[f];
  // ray with unit forward component: a point at depth t is pos + t * d
  const float x = (px + 0.5f - 0.5f * W) / c.fpx, y = -(py + 0.5f - 0.5f * H) / c.fpx;
  float d[3];
#pragma unroll
  for (int i = 0; i < 3; i++) d[i] = c.fwd[i] + x * c.right[i] + y * c.up[i];
  const float dn = sqrtf(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
  float col[3];
  float t_floor = INFINITY;
  if (env.floor_on && d[2] < 0.0f) {
    const float t = (env.floor_z - c.pos[2]) / d[2];
    if (t > NEAR) t_floor = t;
  }
  const unsigned long long z = zbuf[idx];
  const float tz = z == EMPTY ? INFINITY : __uint_as_float((uint32_t)(z >> 32));
  if (tz < t_floor) {
    const uint32_t rgb = (uint32_t)z;
#pragma unroll
    for (int i = 0; i < 3; i++) out[3 * idx + i] = (uint8_t)((rgb >> (8 * i)) & 0xFFu);
    return;
  }
  if (t_floor < INFINITY) {
    const float hx = c.pos[0] + t_floor * d[0], hy = c.pos[1] + t_floor * d[1];
    const int chk = ((int)floorf(hx / env.check) + (int)floorf(hy / env.check)) & 1;
    const float sh = fminf(env.ambient + env.diffuse * (-d[2] / dn), 1.0f);
#pragma unroll
    for (int i = 0; i < 3; i++) col[i] = (chk ? env.floor_rgb1[i] : env.floor_rgb2[i]) * sh;
  } else {
    const float e = 0.5f * (d[2] / dn + 1.0f);  // elevation 0 (down) .. 1 (up)
#pragma unroll
    for (int i = 0; i < 3; i++) col[i] = env.sky_bottom[i] + e * (env.sky_top[i] - env.sky_bottom[i]);
  }
#pragma unroll
  for (int i = 0; i < 3; i++) out[3 * idx + i] = (uint8_t)(fminf(fmaxf(col[i], 0.0f), 1.0f) * 255.0f + 0.5f);
}

}  // namespace pp3r

static thread_local std::string g_render_err;
#define RCHK(x)                                                                  \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      g_render_err = std::string(#x) + ": " + hipGetErrorString(e_);             \
      return PP3_ERR_HIP;                                                        \
    }                                                                            \
  } while (0)

extern "C" {

const char* pp3_render_last_error(void) { return g_render_err.c_str(); }

int pp3_render(int32_t device, const float* tris, const int32_t* tri_geom, int32_t ntri, const float* geom_rgb,
               int32_t ngeom, const float* geom_xf, const float* cams, int32_t nframes, int32_t height, int32_t width,
               const float* scene, uint8_t* out, void* stream) {
  if (!geom_xf || !cams || !scene || !out || nframes <= 0 || height <= 0 || width <= 0 || ngeom <= 0 || ntri < 0 ||
      (ntri > 0 && (!tris || !tri_geom || !geom_rgb))) {
    g_render_err = "pp3_render: invalid argument";
    return PP3_ERR_ARG;
  }
  if (nframes > 65535) {
    g_render_err = "pp3_render: at most 65535 frames per call";
    return PP3_ERR_ARG;
  }
  RCHK(hipSetDevice(device));
  hipStream_t s = (hipStream_t)stream;
  pp3r::Env env;
  memcpy(env.floor_rgb1, scene + 0, 3 * sizeof(float));
  memcpy(env.floor_rgb2, scene + 3, 3 * sizeof(float));
  env.check = scene[6];
  env.floor_z = scene[7];
  memcpy(env.sky_top, scene + 8, 3 * sizeof(float));
  memcpy(env.sky_bottom, scene + 11, 3 * sizeof(float));
  env.ambient = scene[14];
  env.diffuse = scene[15];
  env.floor_on = scene[16] != 0.0f;
  env.pad = 0;
  const size_t npix = (size_t)nframes * height * width;
  unsigned long long* zbuf = nullptr;
  RCHK(hipMalloc(&zbuf, npix * sizeof(unsigned long long)));
  hipError_t err = hipMemsetAsync(zbuf, 0xFF, npix * sizeof(unsigned long long), s);
  if (err == hipSuccess && ntri > 0) {
    hipLaunchKernelGGL(pp3r::raster_kernel, dim3((ntri + 63) / 64, nframes), dim3(64), 0, s, tris, tri_geom, ntri,
                       geom_rgb, geom_xf, ngeom, (const pp3r::Cam*)cams, height, width, env.ambient, env.diffuse, zbuf);
    err = hipGetLastError();
  }
  if (err == hipSuccess) {
    hipLaunchKernelGGL(pp3r::resolve_kernel, dim3((unsigned)((npix + 255) / 256)), dim3(256), 0, s, zbuf,
                       (const pp3r::Cam*)cams, nframes, height, width, env, out);
    err = hipGetLastError();
  }
  if (err == hipSuccess) err = hipStreamSynchronize(s);
  hipError_t ferr = hipFree(zbuf);
  if (err != hipSuccess) {
    g_render_err = std::string("pp3_render: ") + hipGetErrorString(err);
    return PP3_ERR_HIP;
  }
  if (ferr != hipSuccess) {
    g_render_err = std::string("pp3_render: hipFree: ") + hipGetErrorString(ferr);
    return PP3_ERR_HIP;
  }
  return PP3_OK;
}

}  // extern "C"
