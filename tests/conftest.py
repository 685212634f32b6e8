"""pytest configuration: markers, build of the libraries, shared fixtures.

`-m "not gpu"`: oracle vs golden vectors, host logic, C-ABI exports (no GPU).
`-m gpu`: parity of the HIP path (through the C-ABI) against the oracle.
"""
import json
import os
import subprocess
import sys
import time

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "qwen3-asr.cpp_amd", "python"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path)")
    config.addinivalue_line("markers", "slow: long-running (full-size model)")


def _stale(target: str, src_globs) -> bool:
    import glob
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(f) > t for g in src_globs for f in glob.glob(os.path.join(ROOT, g)))


@pytest.fixture(scope="session")
def built():
    """the in-tree libraries, rebuilt (make) when missing or older than any
    source they are built from -- a stale binary never passes silently"""
    lib = os.path.join(ROOT, "qwen3-asr.cpp_amd", "libqasr.so")
    if _stale(lib, ["qwen3-asr.cpp_amd/csrc/*", "qwen3-asr.cpp_amd/host/*", "include/*.h"]):
        subprocess.run(["make", "-s", "-j8", "-C", os.path.join(ROOT, "qwen3-asr.cpp_amd")], check=True)
    orc = os.path.join(ROOT, "oracle", "liboracle.so")
    if not os.path.exists(orc):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    return True


@pytest.fixture(scope="session")
def tiny_gguf(built, tmp_path_factory):
    import qasr
    p = str(tmp_path_factory.mktemp("models") / "tiny-f16.gguf")
    qasr.write_synthetic_gguf(p, "tiny", 42, 1)
    return p


@pytest.fixture(scope="session")
def full_f16_gguf(built, tmp_path_factory):
    """the Qwen3-ASR-0.6B-shaped synthetic f16 GGUF (seed 42), or $QASR_MODEL"""
    import qasr
    if os.environ.get("QASR_MODEL"):
        return os.environ["QASR_MODEL"]
    p = str(tmp_path_factory.mktemp("full") / "full-f16.gguf")
    qasr.write_synthetic_gguf(p, "full", 42, 1)
    return p


@pytest.fixture(scope="session")
def full_q8_gguf(built, tmp_path_factory):
    """the Qwen3-ASR-0.6B-shaped synthetic Q8_0 GGUF (seed 42; configs[2]'s weights)"""
    import qasr
    p = str(tmp_path_factory.mktemp("fq8") / "full-q8.gguf")
    qasr.write_synthetic_gguf(p, "full", 42, 8)
    return p


@pytest.fixture(scope="session")
def tiny_oracle(tiny_gguf):
    import oracle_py as op
    op.set_threads(min(8, os.cpu_count() or 1))
    return op.OracleModel(tiny_gguf)


@pytest.fixture(scope="session")
def tiny_q8_gguf(built, tmp_path_factory):
    """Same seed as tiny_gguf, linear weights Q8_0 (convert_hf_to_gguf.py --type q8_0 policy)."""
    import qasr
    p = str(tmp_path_factory.mktemp("models") / "tiny-q8_0.gguf")
    qasr.write_synthetic_gguf(p, "tiny", 42, 8)
    return p


@pytest.fixture(scope="session")
def tiny_q8_oracle(tiny_q8_gguf):
    import oracle_py as op
    op.set_threads(min(8, os.cpu_count() or 1))
    return op.OracleModel(tiny_q8_gguf)


def gpu_available() -> bool:
    try:
        import qasr
        return qasr.device_count() > 0
    except Exception:
        return False


@pytest.fixture(scope="session")
def gpu(built):
    if not gpu_available():
        pytest.fail("GPU tests need a HIP device: the HIP path has no CPU fallback")
    return True


# ------------------------------------------------------------ parity record
# Every GPU parity test records what it measured (absolute and relative max
# |delta| against the oracle, margins, noise floors) through the `parity`
# fixture; the session writes them to $QASR_PARITY_OUT (default
# gpurun_out/parity.json), which tools/r4 copies to profiles/<round>/parity.json.
_PARITY = {}


def _plain(v):
    if isinstance(v, (list, tuple)):
        return [_plain(x) for x in v]
    if isinstance(v, (np.floating, float)):
        return float(f"{float(v):.6g}")
    if isinstance(v, (np.integer, int)) and not isinstance(v, bool):
        return int(v)
    return v


@pytest.fixture(scope="session")
def parity():
    def rec(name: str, **vals):
        _PARITY.setdefault(name, {}).update({k: _plain(v) for k, v in vals.items()})
    return rec


def pytest_sessionfinish(session, exitstatus):
    if not _PARITY:
        return
    out = os.environ.get("QASR_PARITY_OUT") or os.path.join(ROOT, "gpurun_out", "parity.json")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    env = {k: v for k, v in os.environ.items() if k.startswith("QASR_") and k != "QASR_PARITY_OUT"}
    with open(out, "w") as f:
        json.dump({"written": time.strftime("%Y-%m-%d %H:%M:%S"), "exitstatus": int(exitstatus), "env": env,
                   "tests": dict(sorted(_PARITY.items()))}, f, indent=1)
