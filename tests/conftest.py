import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs via gpurun)")


def pytest_sessionstart(session):
    """Build provenance (verdict r04 #7): the prebuilt libvr.so / libvr_shard.so
    must be built from the checked-out sources -- their embedded build id
    (vr_build_id, vr_shard_build_id) equals tools/build_id.py's hash of
    csrc/ and include/.  A stale library stops the run before any test."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from build_id import build_id
    from volumetricrenderer_amd import _lib
    want = build_id()
    got = {"libvr.so": _lib.load().vr_build_id().decode(),
           "libvr_shard.so": _lib.load_shard().vr_shard_build_id().decode()}
    print(f"\nbuild id of the sources {want}; " + ", ".join(f"{k} {v}" for k, v in got.items()))
    bad = {k: v for k, v in got.items() if v.split("-")[0] != want}
    if bad:
        pytest.exit(f"stale native libraries {bad}: the sources hash to {want} (rebuild: make -C "
                    "volumetricrenderer_amd/csrc)", returncode=3)


@pytest.fixture(scope="session")
def oracle():
    import vr_oracle
    vr_oracle.lib()
    return vr_oracle
