"""tools/png_writer.hpp (the offscreen driver's output path, SURVEY.md sec. 8
f3) round-trips through an independent PNG decoder (PIL): a small C++ harness
is compiled with g++ and writes a known RGBA8 pattern, including sizes whose
rows do not fill a deflate block evenly."""
import os
import shutil
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

HARNESS = r'''
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "png_writer.hpp"
int main(int argc, char** argv) {
    int w = std::atoi(argv[1]), h = std::atoi(argv[2]);
    std::vector<unsigned char> px((size_t)w * h * 4);
    for (size_t i = 0; i < px.size(); ++i) px[i] = (unsigned char)((i * 2654435761u) >> 13);
    return vr::tools::WritePng(argv[3], px.data(), w, h) ? 0 : 1;
}
'''


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
@pytest.mark.parametrize("w,h", [(1, 1), (17, 5), (256, 256), (1000, 70)])
def test_png_writer_roundtrip(tmp_path, w, h):
    src = tmp_path / "h.cpp"
    src.write_text(HARNESS)
    exe = tmp_path / "h"
    subprocess.run(["g++", "-O1", "-std=c++17", "-I", os.path.join(ROOT, "tools"), str(src), "-o", str(exe)],
                   check=True)
    out = tmp_path / "p.png"
    subprocess.run([str(exe), str(w), str(h), str(out)], check=True)
    from PIL import Image
    img = np.asarray(Image.open(out).convert("RGBA"))
    i = np.arange(w * h * 4, dtype=np.uint64)
    want = (((i * np.uint64(2654435761)) & np.uint64(0xFFFFFFFF)) >> np.uint64(13)).astype(np.uint8)
    assert np.array_equal(img.reshape(-1), want)
