"""The north_star's thin C++ host: tools/vr_offscreen (built by
__graft_entry__.build(), replaces the TestMain.cpp:173-256 frame loop) renders
through libvr's C ABI and writes a PNG (tools/png_writer.hpp; the reference
presents to an sRGB swapchain instead, VulkanSwapchain.cpp:181-191).  The
decoded PNG must equal the oracle's RGBA8 frame: bit-exact for UNORM, <= 1 LSB
for sRGB (powf differs between libm and the device library)."""
import os
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tools", "vr_offscreen")


def run_offscreen(tmp_path, W, H, steps, size, fmt, phi=0.0):
    assert os.path.exists(BIN), "tools/vr_offscreen is not built (__graft_entry__.build())"
    out = str(tmp_path / f"f_{W}x{H}_{fmt}.png")
    p = subprocess.run([BIN, "--width", str(W), "--height", str(H), "--steps", str(steps), "--size", str(size),
                        "--frames", "3", "--format", fmt, "--phi", str(phi), "--out", out],
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr
    from PIL import Image
    img = np.asarray(Image.open(out).convert("RGBA"))
    assert img.shape == (H, W, 4)
    return img, p.stdout


def oracle_frame(oracle, W, H, steps, size, fmt, phi=0.0):
    s = np.float32(128.0) / np.float32(size)
    freq = [float(np.float32(f) * s) for f in (0.01, 0.03, 0.19, 0.15)]
    vol = oracle.build_volume(size, freq=freq)
    obj, glob = oracle.reference_shader_data(float(np.float32(W) / np.float32(H)), phi)
    ref, _ = oracle.render(vol, obj, glob, oracle.march(steps), W, H, fmt)
    return ref


@pytest.mark.parametrize("W,H,steps,size", [(256, 256, 32, 64), (1280, 720, 128, 128)])
def test_offscreen_png_unorm_bitexact(tmp_path, oracle, W, H, steps, size):
    img, log = run_offscreen(tmp_path, W, H, steps, size, "unorm")
    ref = oracle_frame(oracle, W, H, steps, size, oracle.FMT_RGBA8_UNORM)
    assert np.array_equal(img, ref), f"{(img != ref).any(axis=2).sum()} pixels differ"
    assert "Mray/s" in log


def test_offscreen_png_srgb(tmp_path, oracle):
    W, H = 640, 360
    img, _ = run_offscreen(tmp_path, W, H, 128, 64, "srgb", phi=30.0)
    ref = oracle_frame(oracle, W, H, 128, 64, oracle.FMT_RGBA8_SRGB, phi=30.0)
    assert np.abs(img.astype(int) - ref.astype(int)).max() <= 1
