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
