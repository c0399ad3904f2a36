"""Where the deferred shadow pass's lane-slots go (config 3, 1080p x 128, 8
sun samples), from the step counter of three builds run in turn:

    libvr.so                        count 1: primary steps + in-box shadow evaluations (V)
    VR_COUNT_SLOTS=1 (libvr_slots1) count 1: primary steps + 8 x entries (E)
    VR_COUNT_SLOTS=2 (libvr_slots2) count 1: primary steps + 512 x chunks (C)

(make -C volumetricrenderer_amd/csrc OUT=../libvr_slotsN.so OBJDIR=/tmp/obj_slotsN
EXTRA=-DVR_COUNT_SLOTS=N ../libvr_slotsN.so).  V / 8E is the in-box share of an
entry's samples, 8E / 512C the chunk fill.

    python tools/shadow_slots.py            # runs the three builds as child processes
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child():
    sys.path.insert(0, ROOT)
    import torch
    import volumetricrenderer_amd as vr
    W, H = 1920, 1080
    r = vr.Renderer(0)
    r.set_procedural(shadow_steps=8)
    r.set_shader_data(*vr.reference_shader_data(1280.0 / 720.0))
    r.set_march(vr.march_defaults(max_steps=128))
    out = {}
    for count in (0, 1):
        r.set_option("count", count)
        cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
        r.render(W, H, vr.FMT_RGBA8_UNORM)   # the sort and the scratch sized
        r.render(W, H, vr.FMT_RGBA8_UNORM, step_counter=cnt)
        torch.cuda.synchronize()
        out[count] = int(cnt.item())
    print(json.dumps(out))


def main():
    res = {}
    for name in ("libvr.so", "libvr_slots1.so", "libvr_slots2.so"):
        env = dict(os.environ, VR_LIB=os.path.join(ROOT, "volumetricrenderer_amd", name))
        p = subprocess.run([sys.executable, __file__, "--child"], env=env, capture_output=True, text=True, timeout=300)
        if p.returncode:
            print(p.stdout, p.stderr)
            sys.exit(p.returncode)
        res[name] = json.loads(p.stdout.strip().splitlines()[-1])
    P = res["libvr.so"]["0"]
    V = res["libvr.so"]["1"] - P
    E8 = res["libvr_slots1.so"]["1"] - res["libvr_slots1.so"]["0"]
    C512 = res["libvr_slots2.so"]["1"] - res["libvr_slots2.so"]["0"]
    print(f"primary steps {P}, shadow evaluations V {V}, entries E {E8 // 8}, chunks C {C512 // 512}")
    print(f"in-box share of the entries' samples V / 8E = {V / E8:.3f}; chunk fill 8E / 512C = {E8 / C512:.3f}; "
          f"lane-slot use V / 512C = {V / C512:.3f}")


if __name__ == "__main__":
    child() if "--child" in sys.argv else main()
