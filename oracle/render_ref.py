"""CPU restatement of csrc/pp3_render.hip (TEST INFRASTRUCTURE ONLY: the checker of
tests/test_gpu_render.py, never imported by the product path).

Same rules in float32 numpy: per (triangle, frame) the transform, pinhole projection, headlight
shade and u8 colour rounding, pixel centres inside all three edge functions (inclusive),
perspective-correct depth, nearest fragment by the (depth bits << 32 | rgb) key; per pixel the
fragment, else the checker floor, else the gradient sky.  Pixels on triangle edges can differ
from the GPU by rounding (fused multiply-adds), so the test compares pixel fractions.
"""
import numpy as np

NEAR = np.float32(1e-3)


def _edge(ax, ay, bx, by, px, py):
    return (bx - ax) * (py - ay) - (by - ay) * (px - ax)


def raster(tris, owner, rgb, xf, cam, H, W, ambient, diffuse):
    f32 = np.float32
    key = np.full((H, W), np.uint64(0xFFFFFFFFFFFFFFFF), np.uint64)
    pos, right, up, fwd, fpx = cam[0:3], cam[3:6], cam[6:9], cam[9:12], cam[12]
    for t in range(len(tris)):
        g = owner[t]
        R = xf[g, :9].reshape(3, 3)
        T = xf[g, 9:]
        v = tris[t].reshape(3, 3)
        w = (v @ R.T + T).astype(f32)
        r = (w - pos).astype(f32)
        cc = np.stack([r @ right, r @ up, r @ fwd], 1).astype(f32)
        if np.any(cc[:, 2] < NEAR):
            continue
        n = np.cross(w[1] - w[0], w[2] - w[0]).astype(f32)
        nn = f32(np.sqrt(f32(n @ n)))
        if nn <= 0:
            continue
        lam = f32(abs(f32(n @ fwd)) / nn)
        sh = min(f32(ambient + diffuse * lam), f32(1.0))
        col = 0
        for i in range(3):
            c = min(max(f32(rgb[g, i] * sh), f32(0)), f32(1))
            col |= int(f32(c * f32(255.0)) + f32(0.5)) << (8 * i)
        sx = (f32(0.5 * W) + fpx * cc[:, 0] / cc[:, 2]).astype(f32)
        sy = (f32(0.5 * H) - fpx * cc[:, 1] / cc[:, 2]).astype(f32)
        area = f32(_edge(sx[0], sy[0], sx[1], sy[1], sx[2], sy[2]))
        if abs(area) < 1e-12:
            continue
        ia = f32(1.0) / area
        x0, x1 = max(0, int(np.floor(sx.min()))), min(W - 1, int(np.ceil(sx.max())))
        y0, y1 = max(0, int(np.floor(sy.min()))), min(H - 1, int(np.ceil(sy.max())))
        if x0 > x1 or y0 > y1:
            continue
        fy, fx = np.meshgrid(np.arange(y0, y1 + 1, dtype=f32) + f32(0.5), np.arange(x0, x1 + 1, dtype=f32) + f32(0.5),
                             indexing="ij")
        b0 = _edge(sx[1], sy[1], sx[2], sy[2], fx, fy).astype(f32) * ia
        b1 = _edge(sx[2], sy[2], sx[0], sy[0], fx, fy).astype(f32) * ia
        b2 = _edge(sx[0], sy[0], sx[1], sy[1], fx, fy).astype(f32) * ia
        inside = (b0 >= 0) & (b1 >= 0) & (b2 >= 0)
        if not inside.any():
            continue
        iz = (f32(1.0) / cc[:, 2]).astype(f32)
        depth = (f32(1.0) / (b0 * iz[0] + b1 * iz[1] + b2 * iz[2])).astype(f32)
        k = (depth.view(np.uint32).astype(np.uint64) << np.uint64(32)) | np.uint64(col)
        sub = key[y0:y1 + 1, x0:x1 + 1]
        np.copyto(sub, np.minimum(sub, k), where=inside)
    return key


def resolve(key, cam, H, W, sp):
    f32 = np.float32
    pos, right, up, fwd, fpx = cam[0:3], cam[3:6], cam[6:9], cam[9:12], cam[12]
    py, px = np.meshgrid(np.arange(H, dtype=f32), np.arange(W, dtype=f32), indexing="ij")
    x = (px + f32(0.5) - f32(0.5 * W)) / fpx
    y = -(py + f32(0.5) - f32(0.5 * H)) / fpx
    d = fwd[None, None] + x[..., None] * right[None, None] + y[..., None] * up[None, None]
    dn = np.sqrt((d * d).sum(-1)).astype(f32)
    rgb1, rgb2, check, fz = sp[0:3], sp[3:6], sp[6], sp[7]
    top, bot, amb, dif, fon = sp[8:11], sp[11:14], sp[14], sp[15], sp[16]
    with np.errstate(divide="ignore", invalid="ignore"):
        t = ((fz - pos[2]) / d[..., 2]).astype(f32)
    hit = (fon != 0) & (d[..., 2] < 0) & (t > NEAR)
    tf = np.where(hit, t, np.inf).astype(f32)
    empty = key == np.uint64(0xFFFFFFFFFFFFFFFF)
    tz = np.where(empty, np.inf, (key >> np.uint64(32)).astype(np.uint32).view(np.float32)).astype(f32)
    out = np.zeros((H, W, 3), np.uint8)
    tri = tz < tf
    c = (key & np.uint64(0xFFFFFF)).astype(np.uint32)
    for i in range(3):
        out[..., i] = np.where(tri, (c >> (8 * i)) & 0xFF, 0)
    hx = pos[0] + tf * d[..., 0]
    hy = pos[1] + tf * d[..., 1]
    with np.errstate(invalid="ignore"):
        chk = (np.floor(hx / check).astype(np.int64) + np.floor(hy / check).astype(np.int64)) & 1
    sh = np.minimum(amb + dif * (-d[..., 2] / dn), f32(1))
    e = f32(0.5) * (d[..., 2] / dn + f32(1))
    for i in range(3):
        floor_c = np.where(chk == 1, rgb1[i], rgb2[i]) * sh
        sky_c = bot[i] + e * (top[i] - bot[i])
        col = np.where(np.isfinite(tf), floor_c, sky_c)
        v = (np.clip(col, 0, 1) * f32(255) + f32(0.5)).astype(np.int64).astype(np.uint8)
        out[..., i] = np.where(tri, out[..., i], v)
    return out


def render(scene, qposes, camera, H, W):
    """Frames [H, W, 3] u8 for the same inputs as pupperv3_mjx.render.render_qpos."""
    sp = scene.scene_params()
    frames = []
    for q in qposes:
        xf = scene.transforms(q)
        cam = scene.camera(camera, q, H)
        key = raster(scene.tris, scene.tri_owner, scene.rgb, xf, cam, H, W, sp[14], sp[15])
        frames.append(resolve(key, cam, H, W, sp))
    return frames
