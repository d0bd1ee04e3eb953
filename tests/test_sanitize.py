"""Host-side AddressSanitizer + UndefinedBehaviorSanitizer build of the C ABI: the search's work-plan,
workspace-sizing and argument-check code (host C++ in the .hip files — round 2's memory fault came from a workspace
size mismatch there) driven by tests/sanitize/plan_check.cpp over the BASELINE configs' query counts and table sizes
and every plan override, in every first-pass geometry.  Device code is compiled normally and never launched; the
sanitizers instrument the host side only (-Xarch_host -fsanitize=...).  CPU only."""
import hashlib
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "audio-compression_amd", "csrc")
OUT = os.path.join(CSRC, "build", "sanitize")
DRIVER = os.path.join(ROOT, "tests", "sanitize", "plan_check.cpp")
SAN = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined"]
FLAGS = ["--offload-arch=gfx950", "-O1", "-g", "-std=c++17", "-fPIC", "-ffp-contract=off", "-DFWAV_DEBUG_API",
         "-fno-omit-frame-pointer", *SAN]


def _build() -> str:
    from fwav import _digest
    key = hashlib.sha256((_digest.source_digest() + open(DRIVER).read() + " ".join(FLAGS)).encode()).hexdigest()
    exe = os.path.join(OUT, "plan_check")
    stamp = exe + ".key"
    if os.path.exists(exe) and os.path.exists(stamp) and open(stamp).read() == key:
        return exe
    os.makedirs(OUT, exist_ok=True)
    srcs = [os.path.join(CSRC, f) for f in sorted(os.listdir(CSRC)) if f.endswith(".hip")]
    procs, objs = [], []
    for s in srcs + [DRIVER]:
        o = os.path.join(OUT, os.path.basename(s).rsplit(".", 1)[0] + ".o")
        objs.append(o)
        lang = ["-x", "hip"] if s.endswith(".cpp") else []
        procs.append(subprocess.Popen(["hipcc", *FLAGS, *lang, "-c", s, "-o", o], stderr=subprocess.PIPE))
    errs = [p.communicate()[1] for p in procs]
    assert all(p.returncode == 0 for p in procs), b"\n".join(errs).decode(errors="replace")[-4000:]
    subprocess.check_call(["hipcc", "--offload-arch=gfx950", *SAN, *objs, "-o", exe])
    with open(stamp, "w") as f:
        f.write(key)
    return exe


@pytest.mark.skipif(shutil.which("hipcc") is None, reason="hipcc not available")
def test_host_plan_and_argument_checks_under_asan_ubsan():
    exe = _build()
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0:exitcode=23",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1:exitcode=24")
    r = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=600)
    print(r.stdout[-2000:], r.stderr[-4000:])
    assert r.returncode == 0, r.stderr[-4000:]
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr
    assert "0 failures" in r.stdout and "default plans covered" in r.stdout
