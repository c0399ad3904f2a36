"""Generate the committed golden fixtures in tests/golden/ from the CPU oracle.

The reference cannot be run here, so these fixtures pin
the oracle against regressions.  They are not reference outputs.  They are
regenerated only deliberately:

    python tests/golden/make_golden.py

Fixtures:
  config1_256x256x32.npy   grey channel (float32) of BASELINE config 1: 256x256,
                           32 steps, aspect 1, single-octave Perlin cube
  config1_256x256x32.png   the same frame as RGBA8 UNORM (for viewing)
  volume16_literal.npy     16^3 RGBA8 volume of the TestMain.cpp:43-92 recipe
  noise_kat.json           noise values at fixed points, per generator
  config2_crop64.npy       grey channel (float32) of a 64x64 crop of BASELINE
                           config 2 (procedural cloud, 1920x1080x128): rows
                           512-575 (band 8 of 64-row bands), cols 928-991
  config3_crop64.npy       the same crop of config 3 (+ 8 shadow steps)
"""
import json
import os
import struct
import sys
import zlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import vr_oracle as oracle  # noqa: E402


def perlin_cube_volume(n=128):
    """Config 1 volume: Perlin f=.19 seed 3, normalised + inverted like
    TestMain.cpp:64-78, the same bytes in all four channels."""
    g, mn, mx = oracle.noise_grid(oracle.NOISE_PERLIN, n, n, n, 0.19, 3)
    inv = np.float32(1.0) / (np.float32(mx) - np.float32(mn))
    s = (np.float32(1.0) - (g - np.float32(mn)) * inv).astype(np.float32)
    b = (s * np.float32(255.0)).astype(np.int32).astype(np.uint8)
    return np.repeat(b[..., None], 4, axis=3)


def write_png(path, rgba):
    h, w, _ = rgba.shape
    raw = b"".join(b"\x00" + rgba[y].tobytes() for y in range(h))

    def chunk(t, d):
        return struct.pack(">I", len(d)) + t + d + struct.pack(">I", zlib.crc32(t + d) & 0xFFFFFFFF)

    png = b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, 6, 0, 0, 0))
    png += chunk(b"IDAT", zlib.compress(raw, 9)) + chunk(b"IEND", b"")
    with open(path, "wb") as f:
        f.write(png)


CROP_BAND = dict(band_rows=64, band_stride=1000, band_first=8)   # rows 512..575 only
CROP_COLS = (928, 992)


def procedural(shadow_steps):
    """vr_procedural_defaults (include/vr.h) with enabled = 1."""
    p = oracle.Procedural()
    p.enabled, p.grid_scale, p.octaves, p.freq0, p.lacunarity, p.gain = 1, 128.0, 4, 0.19, 2.0, 0.5
    p.seed_fbm, p.worley_freq, p.seed_worley, p.shadow_steps = 3, 0.03, 2, shadow_steps
    n = (1.0 + 1.0 + 4.0) ** 0.5
    p.sun_dir[:] = [float(np.float32(1.0 / n)), float(np.float32(1.0 / n)), float(np.float32(2.0 / n))]
    return p


def procedural_crop(shadow_steps):
    obj, glob = oracle.reference_shader_data(1280.0 / 720.0)
    img, _ = oracle.render_procedural(oracle.procedural_from(procedural(shadow_steps)), obj, glob, oracle.march(128),
                                      1920, 1080, oracle.FMT_RGBA32F, **CROP_BAND)
    return img[:, CROP_COLS[0]:CROP_COLS[1], 0].astype(np.float32)


NOISE_POINTS = [(0.0, 0.0, 0.0), (0.5, 0.25, 0.125), (1.3, -2.7, 5.9), (12.34, 56.78, -9.1),
                (-100.5, 33.3, 0.001), (127.0 * 0.19, 3.0 * 0.19, 64.0 * 0.19), (1e3, -1e3, 0.5)]


def main():
    vol = perlin_cube_volume()
    obj, glob = oracle.reference_shader_data(1.0)
    img, steps = oracle.render(vol, obj, glob, oracle.march(32), 256, 256, oracle.FMT_RGBA32F)
    np.save(os.path.join(HERE, "config1_256x256x32.npy"), img[..., 0].astype(np.float32))
    img8, _ = oracle.render(vol, obj, glob, oracle.march(32), 256, 256, oracle.FMT_RGBA8_UNORM)
    write_png(os.path.join(HERE, "config1_256x256x32.png"), img8)
    np.save(os.path.join(HERE, "volume16_literal.npy"), oracle.build_volume(16))
    L = oracle.lib()
    kat = {"points": NOISE_POINTS, "config1_steps": steps}
    for name, f in (("perlin", L.vro_perlin3), ("simplex", L.vro_simplex3), ("cellular", L.vro_cellular3)):
        kat[name] = {str(seed): [float(np.float32(f(seed, *p))) for p in NOISE_POINTS] for seed in (1, 2, 3, 1337)}
    with open(os.path.join(HERE, "noise_kat.json"), "w") as fh:
        json.dump(kat, fh, indent=1)
    np.save(os.path.join(HERE, "config2_crop64.npy"), procedural_crop(0))
    np.save(os.path.join(HERE, "config3_crop64.npy"), procedural_crop(8))
    print("wrote fixtures; config-1 executed steps", steps)


if __name__ == "__main__":
    main()
