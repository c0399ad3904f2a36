"""The build id of libvr.so / libvr_shard.so: a hash of the sources they are
built from (volumetricrenderer_amd/csrc: *.hip, *.cpp, *.h, Makefile;
include/: *.h, *.hpp).  The Makefile embeds it (vr_build_id(),
vr_shard_build_id()); tests/conftest.py and __graft_entry__.smoke() compare
it with the checked-out sources, so a stale prebuilt library cannot pass for
HEAD's code.

    python3 tools/build_id.py          # prints the id
"""
import hashlib
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DIRS = {os.path.join("volumetricrenderer_amd", "csrc"): (".hip", ".cpp", ".h", "Makefile"),
        "include": (".h", ".hpp")}


def source_files():
    out = []
    for d, exts in DIRS.items():
        for name in sorted(os.listdir(os.path.join(ROOT, d))):
            p = os.path.join(d, name)
            if os.path.isfile(os.path.join(ROOT, p)) and name.endswith(exts):
                out.append(p)
    return sorted(out)


def build_id() -> str:
    h = hashlib.sha256()
    for p in source_files():
        h.update(p.replace(os.sep, "/").encode() + b"\0")
        with open(os.path.join(ROOT, p), "rb") as f:
            h.update(f.read() + b"\0")
    return h.hexdigest()[:16]


if __name__ == "__main__":
    print(build_id())
