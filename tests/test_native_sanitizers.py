"""The threaded C++ control plane (``_native``: search methods, scheduler, the std::thread record
loader) under AddressSanitizer+UBSan and ThreadSanitizer (the reference runs its Go tests under
``-race``).  Builds the instrumented copy (``python -m determined_amd._build --sanitize <kind>``) and
re-runs the native test files in a subprocess with the sanitizer runtime preloaded; any report fails
the run (ASan/UBSan/TSan halt on the first error)."""

import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TESTS = ["tests/test_native_loader.py", "tests/test_scheduler.py", "tests/test_searcher.py",
         "tests/test_searcher_go_vectors.py", "tests/test_scheduler_go_vectors.py"]


@pytest.mark.slow
@pytest.mark.parametrize("kind", ["address", "thread"])
def test_native_tests_pass_under_sanitizer(kind):
    from determined_amd import _build

    so = _build.build_native(sanitize=kind)
    env = dict(os.environ, DAMD_NATIVE_PATH=str(so), LD_PRELOAD=_build.sanitizer_runtime(kind),
               ASAN_OPTIONS="detect_leaks=0:halt_on_error=1:abort_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1",
               TSAN_OPTIONS="halt_on_error=1:second_deadlock_stack=1")
    r = subprocess.run([sys.executable, "-m", "pytest", "-x", "-q", "-p", "no:cacheprovider", "-m", "not gpu", *TESTS],
                       cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=900)
    out = r.stdout
    assert r.returncode == 0, out[-4000:]
    assert "Sanitizer" not in out and "runtime error" not in out, out[-4000:]
    assert " passed" in out
