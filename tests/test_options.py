"""CPU: every per-context option the product reads from the environment
(engine.hip fuse_options(): {"name", "QASR_NAME", ...}) is switched by at
least one GPU test -- a bit-identity or oracle-bar check against the default
-- so no environment variable can move the product onto an unverified path
("remove or test every environment-reachable option")."""
import glob
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _options():
    src = open(os.path.join(ROOT, "qwen3-asr.cpp_amd", "csrc", "engine.hip")).read()
    body = src[src.index("fuse_options()"):]
    body = body[:body.index("return v;")]
    return re.findall(r'\{"([a-z0-9_]+)", "QASR_[A-Z0-9_]+"', body)


def test_every_env_option_has_a_gpu_test():
    opts = _options()
    assert len(opts) >= 20, opts
    text = "".join(open(f).read() for f in glob.glob(os.path.join(ROOT, "tests", "test_gpu_*.py")))
    untested = [o for o in opts
                if f'set_option("{o}"' not in text and f'dict({o}=' not in text and f', {o}=' not in text
                and f'"{o}": (' not in text]
    assert not untested, f"options with no GPU test: {untested}"


# environment variables the product reads outside fuse_options(), each with
# the GPU test that switches it (or why none is needed)
OTHER_ENV = {
    "QASR_NO_GRAPH": "test_gpu_stream.py::test_env_eager_and_trace_paths_equal_default",
    "QASR_DEV_TRACE": "test_gpu_stream.py::test_env_eager_and_trace_paths_equal_default",
    "QASR_DEV_TRACE_LAYER": "test_gpu_stream.py::test_env_eager_and_trace_paths_equal_default",
    "QASR_DEVICE": "device index of the reference-API component objects (no kernel choice); test_refapi.py runs them",
    "QASR_DEV_SKIP": "read only in -DQASR_DIAG_SKIP builds (tools/), never by libqasr.so",
}


def test_every_getenv_is_an_option_or_listed():
    """every getenv("QASR_...") in csrc/ and host/ is a
    fuse_options() entry (tested above) or listed in OTHER_ENV; QASR_DEV_SKIP
    (drops decode kernels) is compiled only into diagnostic builds"""
    src = {}
    for pat in ("csrc/*.hip", "csrc/*.h", "host/*.cpp", "host/*.h"):
        for f in glob.glob(os.path.join(ROOT, "qwen3-asr.cpp_amd", pat)):
            src[f] = open(f).read()
    env = set()
    for text in src.values():
        env |= set(re.findall(r'getenv\("(QASR_[A-Z0-9_]+)"\)', text))
    engine = src[os.path.join(ROOT, "qwen3-asr.cpp_amd", "csrc", "engine.hip")]
    fuse_env = set(re.findall(r'\{"[a-z0-9_]+", "(QASR_[A-Z0-9_]+)"', engine[engine.index("fuse_options()"):]))
    assert env, "no getenv found (pattern drift)"
    unlisted = sorted(env - fuse_env - set(OTHER_ENV))
    assert not unlisted, f"environment variables with no option entry or test: {unlisted}"
    i = engine.index('getenv("QASR_DEV_SKIP")')
    assert engine.rfind("#ifdef QASR_DIAG_SKIP", 0, i) > engine.rfind("#endif", 0, i), "QASR_DEV_SKIP outside its #ifdef"
    tests = "".join(open(f).read() for f in glob.glob(os.path.join(ROOT, "tests", "test_gpu_*.py")))
    for var, why in OTHER_ENV.items():
        if "::" in why:
            assert var in tests, (var, why)


def test_launch_dispatch_has_no_silent_default():
    """launch_gemm / launch_gemv record an unsupported
    (mode, epilogue) pair (note_declined) instead of returning silently"""
    g = open(os.path.join(ROOT, "qwen3-asr.cpp_amd", "csrc", "gemm.hip")).read()
    for fn in ("void launch_gemm(", "void launch_gemv("):
        body = g[g.index(fn):]
        body = body[:body.index("\n}\n")]
        assert "default: break;" not in body, fn
        assert "note_declined" in body, fn
