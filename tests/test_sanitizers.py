"""CPU sanitizer builds of the host negative sampler (race detection).

ncf_amd/csrc/sampler.cpp (+ mt_jump.h) runs the parallel ng_sample pass
(datasets.py:53-69) on a pool of host threads synchronised by hand-rolled spin
barriers and relaxed / acq_rel atomics (sampler.cpp Pool).  Here it is compiled
with -fsanitize=address and with -fsanitize=thread (NCF_SANITIZE: one version of
the multiversioned functions, see mt_jump.h) together with
tests/sanitize/sampler_driver.cpp, which runs two consecutive passes on the
ml-1m-shaped synthetic data set at 2, 8 and 12 threads against the sequential
pass (negatives, word counts, end state) and the parallel MT19937 word generator
against the sequential stream.  The run must be clean under both sanitizers and
its first pass bit-exact against the oracle's C restatement of the reference loop
(oracle/sampler_oracle.c)."""
import os
import shutil
import subprocess

import numpy as np
import pytest

from oracle import ncf_oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "ncf_amd", "csrc")
DRIVER = os.path.join(ROOT, "tests", "sanitize", "sampler_driver.cpp")
THREADS = ["2", "8", "12"]
SAN = {"address": ["-fsanitize=address", "-fno-omit-frame-pointer"], "thread": ["-fsanitize=thread"]}


@pytest.fixture(scope="module")
def ml1m_input(tmp_path_factory):
    from ncf_amd import synthetic
    ds = synthetic.make_dataset("ml-1m", seed=0)
    u = ds["train_users"].astype(np.int32)
    i = ds["train_items"].astype(np.int32)
    path = tmp_path_factory.mktemp("san") / "ml1m.bin"
    with open(path, "wb") as f:
        f.write(np.int64(len(u)).tobytes())
        f.write(np.array([ds["user_num"], ds["item_num"], 4], dtype=np.int32).tobytes())
        f.write(np.uint32(0).tobytes())   # np.random.seed(0)
        f.write(np.int32(2).tobytes())    # two consecutive passes
        f.write(u.tobytes())
        f.write(i.tobytes())
    return path, u, i, int(ds["item_num"])


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
@pytest.mark.parametrize("kind", ["address", "thread"])
def test_sampler_clean_under_sanitizer(kind, ml1m_input, tmp_path):
    path, u, i, n_items = ml1m_input
    exe = str(tmp_path / f"sampler_{kind}")
    subprocess.run(["g++", "-O1", "-g", "-std=c++17", "-DNCF_SANITIZE", "-march=x86-64-v2", "-pthread"] + SAN[kind] +
                   [os.path.join(CSRC, "sampler.cpp"), DRIVER, "-o", exe], check=True, capture_output=True)
    out = str(tmp_path / "neg.bin")
    env = dict(os.environ, ASAN_OPTIONS="verify_asan_link_order=0:detect_leaks=1", TSAN_OPTIONS="halt_on_error=0")
    env.pop("NCF_SAMPLER_THREADS", None)
    p = subprocess.run([exe, str(path), out] + THREADS, capture_output=True, text=True, env=env, timeout=600)
    report = p.stderr[-6000:]
    assert "ThreadSanitizer" not in p.stderr and "AddressSanitizer" not in p.stderr and \
        "LeakSanitizer" not in p.stderr, report
    assert p.returncode == 0, report
    assert "bad 0" in p.stdout and "redone 0" in p.stdout, p.stdout
    neg = np.fromfile(out, dtype=np.int32)
    np.testing.assert_array_equal(neg, O.ng_sample(u, i, n_items, 4, 0))
