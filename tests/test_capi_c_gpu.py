"""The C ABI from a native C caller (tests/capi_c/abi_test.c, built by tfhe-rs-odd_amd/Makefile):
scratch sized only through the *_scratch queries, async PBS / async KS->PBS / submit-wait bit-exact
against the synchronous calls, short or NULL scratch rejected, and context_destroy with a queued
request failing that request (rc = 1) instead of running it on freed state.  The error convention
is the reference C API's (tfhe/src/c_api/utils.rs:3-73)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tfhe-rs-odd_amd", "lib", "abi_test")
SRC = os.path.join(ROOT, "tests", "capi_c", "abi_test.c")


def test_header_compiles_as_c11():
    """include/tfhe_mi355.h is a plain C header: a C11 translation unit using it compiles warning-free."""
    r = subprocess.run(["gcc", "-std=c11", "-Wall", "-Wextra", "-Werror", "-fsyntax-only",
                        "-I", os.path.join(ROOT, "include"), "-I", "/opt/rocm/include", SRC],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def _run(mode, extra_env=None, timeout=300):
    if not os.path.exists(BIN):
        pytest.fail(f"{BIN} is missing: build with `make -C tfhe-rs-odd_amd` (or __graft_entry__.build())")
    env = dict(os.environ)
    env.update(extra_env or {})
    r = subprocess.run([BIN, mode], capture_output=True, text=True, timeout=timeout, env=env)
    print(r.stdout)
    print(r.stderr)
    return r


@pytest.mark.gpu
def test_c_caller_contract():
    r = _run("contract")
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ALL OK" in r.stdout


@pytest.mark.gpu
def test_c_caller_multi_device_context():
    """tfhe_mi355_context_create_devices({0, 0}) from C: every batched / count-1 / submitted call
    bit-identical to a single-device context with the same keys."""
    r = _run("multi")
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ALL OK" in r.stdout


@pytest.mark.gpu
def test_c_caller_destroy_with_queued_request_fails_it():
    # a 2 s coalescing window keeps the submitted request queued until destroy runs
    r = _run("destroy", {"TFHE_MI355_COALESCE_WINDOW_US": "2000000", "TFHE_MI355_COALESCE_GAP_US": "2000000"})
    assert r.returncode == 0, r.stdout + r.stderr
    assert "destroy: rc 1" in r.stdout and "wait: rc 1" in r.stdout
