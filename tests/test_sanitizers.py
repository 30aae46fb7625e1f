"""Host runtime under ThreadSanitizer and AddressSanitizer+UBSan.

The reference has no sanitizer targets and several latent host races (SURVEY
§5.2 list). Here the concurrent host paths (work-stealing CPU threads, the
multi-worker round runner with its watchdog and fault injection, multithreaded
CPU engines) run under both sanitizers with golden checks; any report fails."""
import subprocess

import pytest

from dist_gpu_accelerated_tree_search_amd.ops.build import build_sanitized_selftests


@pytest.fixture(scope="module")
def selftests():
    return build_sanitized_selftests()


@pytest.mark.parametrize("kind", ["tsan", "asan"])
def test_runtime_selftest_clean(selftests, kind):
    env = {"TSAN_OPTIONS": "halt_on_error=1 exitcode=66", "ASAN_OPTIONS": "detect_leaks=1:halt_on_error=1",
           "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1", "PATH": "/usr/bin:/bin"}
    out = subprocess.run([str(selftests[kind])], capture_output=True, text=True, timeout=600, env=env)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-4000:]
    assert "SELFTEST OK" in out.stdout
    assert "WARNING: ThreadSanitizer" not in out.stderr and "ERROR: AddressSanitizer" not in out.stderr
