"""C-ABI checks that need no GPU: the library loads, exports exactly what
include/vr.h declares, and its host-only entry points behave."""
import ctypes
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions(header="vr.h"):
    src = open(os.path.join(ROOT, "include", header)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(vr_[a-z_0-9]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    from volumetricrenderer_amd import _lib
    lib = _lib.load()
    declared = header_functions()
    assert len(declared) >= 20
    for name in declared:
        assert hasattr(lib, name), name
    assert sorted(declared) == _lib.exported_symbols()


def test_shard_library_exports_every_declared_symbol():
    """libvr_shard.so (multi-GPU frame loop, RCCL) loads without a GPU and
    exports exactly what include/vr_shard.h declares."""
    from volumetricrenderer_amd import _lib
    lib = _lib.load_shard()
    declared = header_functions("vr_shard.h")
    assert len(declared) == 36
    for name in declared:
        assert hasattr(lib, name), name
    assert sorted(declared) == _lib.shard_exported_symbols()
    with pytest.raises(_lib.VRError):
        _lib.shard_call("vr_shard_create", None, None, 1, 0, 64, 64, 1, 16, ctypes.byref(ctypes.c_void_p()))
    with pytest.raises(_lib.VRError):   # argument check only, no GPU
        _lib.shard_call("vr_shard_share_volume", None, None, 8, 8, 8, None)
    for bad in (0, 3):   # render streams: 1 or 2
        with pytest.raises(_lib.VRError):
            _lib.shard_call("vr_shard_set_render_streams", None, bad)
    with pytest.raises(_lib.VRError):
        _lib.shard_call("vr_shard_set_solo", None, 1)
    assert _lib.shard_call("vr_shard_get_render_streams", None) == 0
    with pytest.raises(_lib.VRError):
        _lib.shard_call("vr_shard_set_compositor", None, 1)
    with pytest.raises(_lib.VRError):
        _lib.shard_call("vr_shard_bands", None, None, None, None)
    assert _lib.shard_call("vr_shard_get_compositor", None) == -1
    with pytest.raises(_lib.VRError):
        _lib.shard_call("vr_shard_set_serpentine", None, 1)
    assert _lib.shard_call("vr_shard_get_serpentine", None) == -1
    for f, args in (("vr_shard_set_rows", (None, None)), ("vr_shard_balance_rows", (None,)),
                    ("vr_shard_rebalance_rows", (None, 1.0)),
                    ("vr_shard_row_range", (None, 0, None, None))):
        with pytest.raises(_lib.VRError):
            _lib.shard_call(f, *args)
    assert _lib.shard_call("vr_shard_partition", None) == -1


def test_shard_deadline_loop_selftest():
    """The deadline logic every collective wait of libvr_shard uses
    (poll_until), run on the host with stub states: a state that settles, one
    that fails, one that never settles (returns at the deadline, does not
    hang).  Verdict r02 #6: a failing peer must give rc != 0, not a hang."""
    import time
    from volumetricrenderer_amd import _lib
    n = ctypes.c_int()
    assert _lib.shard_call("vr_shard_poll_selftest", 0, 5.0, ctypes.byref(n)) == 0 and n.value == 5
    assert _lib.shard_call("vr_shard_poll_selftest", 1, 5.0, ctypes.byref(n)) == 1 and n.value == 3
    t0 = time.perf_counter()
    assert _lib.shard_call("vr_shard_poll_selftest", 2, 0.05, ctypes.byref(n)) == 2
    el = time.perf_counter() - t0
    assert 0.05 <= el < 2.0 and n.value >= 2
    assert _lib.shard_call("vr_shard_poll_selftest", 3, 0.05, ctypes.byref(n)) == -1
    with pytest.raises(_lib.VRError):
        _lib.shard_call("vr_shard_set_timeout", None, 1.0)
    assert _lib.shard_call("vr_shard_aborted", None) == 0
    # round 6: lead rows and the sampled busy time refuse a null shard
    with pytest.raises(_lib.VRError):
        _lib.shard_call("vr_shard_set_lead_rows", None, 16)
    with pytest.raises(_lib.VRError):
        _lib.shard_call("vr_shard_balance_lead", None, 80)
    assert _lib.shard_call("vr_shard_get_lead_rows", None) == -1
    b, sp = ctypes.c_double(), ctypes.c_double()
    with pytest.raises(_lib.VRError):
        _lib.shard_call("vr_shard_sampled_busy", None, ctypes.byref(b), ctypes.byref(sp))
    assert _lib.STATUS_NAMES[7] == "VR_ERR_TIMEOUT" and _lib.STATUS_NAMES[8] == "VR_ERR_COMM"


def test_volume_extent_ok():
    from volumetricrenderer_amd import _lib
    ok = lambda *d: _lib.call("vr_volume_extent_ok", *d)  # noqa: E731
    assert ok(1, 1, 1) == 1 and ok(512, 512, 512) == 1
    assert ok(0, 4, 4) == 0 and ok(4, -1, 4) == 0 and ok(2000, 2000, 2000) == 0


def test_abi_struct_layouts():
    from volumetricrenderer_amd import _lib
    assert ctypes.sizeof(_lib.ObjectShaderData) == 192
    assert ctypes.sizeof(_lib.GlobalShaderData) == 144
    assert _lib.GlobalShaderData.media_scroll.offset == 80  # std140
    assert ctypes.sizeof(_lib.MarchParams) == 88
    assert ctypes.sizeof(_lib.Target) == 56
    assert _lib.load().vr_abi_version() == 2


def test_no_device_is_a_clean_error():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    import volumetricrenderer_amd as vr
    with pytest.raises(vr.VRError) as e:
        vr.Renderer(0)
    assert e.value.status == 6  # VR_ERR_NO_DEVICE


def test_defaults_are_the_reference_constants():
    import volumetricrenderer_amd as vr
    m = vr.march_defaults()
    assert m.max_steps == 128 and m.step_scale == 4.0 and m.density == 1.0  # frag.glsl:29-30,42
    assert abs(m.scale - 0.2) < 1e-7                                       # :63
    assert list(m.box_min) == [-1, -1, -1] and list(m.box_max) == [1, 1, 1]  # :31-32
    np.testing.assert_allclose(list(m.tap_scale), [1, .8, .75, .7], rtol=1e-7)   # :66-69
    np.testing.assert_allclose(list(m.tap_weight), [0, .2, .25, .3], rtol=1e-7)
    r = vr.volume_recipe_defaults()
    assert r.size == 128 and list(r.seed) == [1, 2, 3, 4] and r.literal_overwrite == 1  # TestMain.cpp:51-62
    np.testing.assert_allclose(list(r.freq), [.01, .03, .19, .15], rtol=1e-7)


@pytest.mark.parametrize("aspect,phi,theta,t", [(16 / 9, 0, 0, 0), (1.0, 30, -20, 1.5), (2.0, 123, 45, 0)])
def test_reference_shader_data_matches_oracle(oracle, aspect, phi, theta, t):
    import volumetricrenderer_amd as vr
    osd, gsd = vr.reference_shader_data(aspect, phi, theta, t)
    obj, glob = vr.shader_data_arrays(osd, gsd)
    o2, g2 = oracle.reference_shader_data(aspect, phi, theta, t)
    assert obj.tobytes() == o2.tobytes()
    assert glob.tobytes() == g2.tobytes()


def test_band_rows_packed():
    import volumetricrenderer_amd as vr
    from volumetricrenderer_amd.distributed import rows_for_rank
    for H in (1, 15, 16, 17, 720, 1080, 2160):
        for n in (1, 2, 3, 8):
            rows = [vr.band_rows_packed(H, 16, n, k) for k in range(n)]
            assert rows == [rows_for_rank(H, 16, n, k) for k in range(n)]
            assert sum(rows) >= H and sum(rows) - H < 16
    assert vr.band_rows_packed(1080, 0, 1, 0) == 1080


def flipped_bands(H, br, stride, first, flip):
    """The frame bands of a band set with its odd bands shifted by flip
    (vr.h vr_target.band_flip), by enumeration."""
    nb, out, k = -(-H // br), [], 0
    while True:
        b = first + k * stride + (flip if k % 2 else 0)
        if b >= nb:
            if first + k * stride >= nb and first + (k + 1) * stride + flip >= nb:
                return out
        else:
            out.append(b)
        k += 1


def test_band_rows_packed_serpentine():
    """vr_band_rows_packed with band_flip: the serpentine deal of S renderers
    (flip S-1-2i) covers every band of the frame exactly once, and each set's
    packed rows are its whole bands; bad flips are refused."""
    import volumetricrenderer_amd as vr
    for H in (16, 17, 100, 720, 1080, 792, 2160):
        for S in (2, 3, 7, 8):
            seen = []
            for i in range(S):
                bands = flipped_bands(H, 16, S, i, S - 1 - 2 * i)
                assert bands == sorted(bands)
                assert vr.band_rows_packed(H, 16, S, i, S - 1 - 2 * i) == 16 * len(bands), (H, S, i)
                seen += bands
            assert sorted(seen) == list(range(-(-H // 16)))
    # an offset set (below a lead of 18 bands) with a negative and a positive flip
    for flip in (-6, -1, 1, 6):
        assert vr.band_rows_packed(1080, 16, 7, 20, flip) == 16 * len(flipped_bands(1080, 16, 7, 20, flip))
    for bad in ((1080, 16, 7, 0, 7), (1080, 16, 7, 0, -7), (1080, 16, 1, 0, 1), (1080, 0, 7, 0, 1)):
        with pytest.raises(ValueError):
            vr.band_rows_packed(*bad)


def test_header_layouts_match_ctypes(tmp_path):
    """Compile include/vr.h with gcc and compare every struct's size (and the
    std140 MediaScroll offset) with the ctypes mirrors."""
    import subprocess
    from volumetricrenderer_amd import _lib
    src = tmp_path / "sizes.c"
    src.write_text(
        '#include <stdio.h>\n#include <stddef.h>\n#include "vr.h"\n'
        "int main(void){printf(\"%zu %zu %zu %zu %zu %zu %zu %zu\\n\","
        "sizeof(vr_object_shader_data), sizeof(vr_global_shader_data),"
        "offsetof(vr_global_shader_data, media_scroll), sizeof(vr_march_params),"
        "sizeof(vr_target), sizeof(vr_volume_recipe), sizeof(vr_procedural), offsetof(vr_procedural, sun_dir));"
        "return 0;}\n")
    exe = tmp_path / "sizes"
    subprocess.run(["gcc", "-std=c99", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    got = [int(v) for v in subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split()]
    want = [ctypes.sizeof(_lib.ObjectShaderData), ctypes.sizeof(_lib.GlobalShaderData),
            _lib.GlobalShaderData.media_scroll.offset, ctypes.sizeof(_lib.MarchParams), ctypes.sizeof(_lib.Target),
            ctypes.sizeof(_lib.VolumeRecipe), ctypes.sizeof(_lib.Procedural), _lib.Procedural.sun_dir.offset]
    assert got == want


def test_procedural_defaults_and_oracle_mirror(oracle):
    import volumetricrenderer_amd as vr
    p = vr.procedural_defaults()
    assert p.enabled == 1 and p.octaves == 4 and p.seed_fbm == 3 and p.seed_worley == 2 and p.shadow_steps == 0
    np.testing.assert_allclose([p.grid_scale, p.freq0, p.lacunarity, p.gain, p.worley_freq],
                               [128, .19, 2, .5, .03], rtol=1e-7)
    np.testing.assert_allclose(list(p.sun_dir), np.array([1, 1, 2]) / np.sqrt(6), rtol=1e-7)
    assert ctypes.sizeof(oracle.Procedural) == ctypes.sizeof(vr.Procedural)
    q = oracle.procedural_from(p)
    assert bytes(q) == bytes(p)   # already unit length: normalising again changes nothing
