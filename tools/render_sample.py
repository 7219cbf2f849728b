"""A few frames of a configs[1] rollout through PupperV3Env.render (tracking_cam, 240 x 320) as
PNG files: python tools/render_sample.py OUT_DIR [meshdir]"""
import os
import struct
import sys
import zlib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pupperv3-mjx_amd")]


def write_png(path, img):
    h, w, _ = img.shape
    raw = b"".join(b"\0" + img[y].tobytes() for y in range(h))

    def chunk(tag, data):
        return struct.pack(">I", len(data)) + tag + data + struct.pack(">I", zlib.crc32(tag + data) & 0xFFFFFFFF)

    with open(path, "wb") as f:
        f.write(b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, 2, 0, 0, 0))
                + chunk(b"IDAT", zlib.compress(raw, 9)) + chunk(b"IEND", b""))


def main():
    import numpy as np
    from bench import bench_kwargs
    from pupperv3_mjx import MODEL_XML
    from pupperv3_mjx.environment import PupperV3Env, make_keys
    out = sys.argv[1]
    meshdir = sys.argv[2] if len(sys.argv) > 2 else None
    os.makedirs(out, exist_ok=True)
    env = PupperV3Env(**bench_kwargs(MODEL_XML), num_envs=1)
    st = env.reset(make_keys(0, 1))
    traj = [st]
    rs = np.random.RandomState(0)
    for _ in range(60):
        st = env.step(st, rs.uniform(-0.5, 0.5, (1, 12)).astype(np.float32))
        traj.append(st)
    frames = env.render(traj[::15], camera="tracking_cam", meshdir=meshdir)
    for i, f in enumerate(frames):
        write_png(os.path.join(out, f"frame_{i:02d}.png"), f)
    env.close()
    print(len(frames), "frames ->", out)


if __name__ == "__main__":
    main()
