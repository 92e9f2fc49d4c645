"""The C-ABI boundary without a GPU: every function include/clearvae.h declares is exported by
libclearvae_hip.so and bound in cvhip/_lib.py, and every struct the binding mirrors has the same size
and field offsets as the C header (checked by compiling a probe against the header with gcc).
Only host-side entry points that never touch the device are called."""

import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "clearvae.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\**\s*(cv_[a-z_0-9]+)\s*\(", src, flags=re.M)))


def test_header_declares_the_hot_path():
    fns = header_functions()
    for need in ("cv_conv_forward", "cv_conv_backward_data", "cv_conv_backward_weight", "cv_linear_forward",
                 "cv_output_loss", "cv_reparam_forward", "cv_latent_combine", "cv_ntxent", "cv_mi_forward",
                 "cv_mi_backward", "cv_mi_learning_step", "cv_adam_step", "cv_last_error", "cv_pack_conv_weights",
                 "cv_latent_step", "cv_step_reduce", "cv_conv_backward_weight_deferred",
                 "cv_linear_backward_weight_deferred", "cv_tc_forward", "cv_tc_learning_step"):
        assert need in fns, need


def test_library_exports_every_declared_symbol():
    from cvhip import _lib

    lib = ctypes.CDLL(_lib.LIB_PATH)
    missing = [f for f in header_functions() if not hasattr(lib, f)]
    assert not missing, missing


def test_binding_covers_header_exactly():
    from cvhip import _lib

    assert sorted(_lib.EXPORTED) == header_functions()


def test_host_only_queries():
    from cvhip import _lib

    L = _lib.lib()
    assert L.cv_version()
    g = _lib.cv_conv(512, 32, 14, 14, 64, 7, 7, 3, 3, 2, 1, 0)
    wb = L.cv_conv_wgrad_workspace_bytes(ctypes.byref(g), 0)
    assert wb > 0 and wb % 4 == 0
    assert L.cv_mi_workspace_bytes(512) > 0


def test_error_path_without_launch():
    """Host-side validation rejects a bad geometry before anything is enqueued."""
    from cvhip import _lib

    L = _lib.lib()
    g = _lib.cv_conv(8, 32, 14, 14, 64, 9, 9, 3, 3, 2, 1, 0)  # wrong output size
    op = _lib.cv_operand(1, None, 0, 0)
    rc = L.cv_conv_forward(ctypes.byref(g), ctypes.byref(op), 1, None, 1, None, None)
    assert rc != 0
    assert b"conv" in L.cv_last_error()


PROBE = r"""
#include <stdio.h>
#include <stddef.h>
#include "clearvae.h"
#define S(T) printf(#T " size %zu\n", sizeof(T));
#define O(T, f) printf(#T " " #f " %zu\n", offsetof(T, f));
int main(void) {
  S(cv_bn) O(cv_bn, stat) O(cv_bn, C) O(cv_bn, eps)
  S(cv_operand) O(cv_operand, xf) O(cv_operand, bn)
  S(cv_epilogue) O(cv_epilogue, stat_out) O(cv_epilogue, ebn) O(cv_epilogue, erelu)
  S(cv_conv) O(cv_conv, transposed) O(cv_conv, mma)
  S(cv_linear) O(cv_linear, out_ch) O(cv_linear, mma)
  S(cv_wgrad_defer) O(cv_wgrad_defer, split) O(cv_wgrad_defer, kk) O(cv_wgrad_defer, gweight) O(cv_wgrad_defer, gbias)
  S(cv_conv_pack) O(cv_conv_pack, cs) O(cv_conv_pack, kw)
  S(cv_ntxent_branch)
  S(cv_mlp) S(cv_mlp_grad)
  S(cv_tc_disc) O(cv_tc_disc, zdim) S(cv_tc_grad)
  return 0;
}
"""


def test_struct_layouts_match_header(tmp_path):
    from cvhip import _lib

    c = tmp_path / "probe.c"
    c.write_text(PROBE)
    exe = tmp_path / "probe"
    r = subprocess.run(["gcc", "-std=c11", "-I", os.path.dirname(HEADER), str(c), "-o", str(exe)],
                       capture_output=True, text=True)
    if r.returncode != 0:
        pytest.fail(r.stderr)
    out = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split("\n")
    for line in filter(None, out):
        parts = line.split()
        T = getattr(_lib, parts[0])
        if parts[1] == "size":
            assert ctypes.sizeof(T) == int(parts[2]), line
        else:
            assert getattr(T, parts[1]).offset == int(parts[2]), line


def test_host_validation_under_asan():
    """`make asan` (SURVEY.md §5 host-side sanitizer build): the library's host code compiled host-only with
    -fsanitize=address, and tests/abi_asan.c driving the C-ABI's validation paths and host-side builders
    against it (no GPU: every call is rejected or answered before a launch).  A failed check or any ASan report
    fails the run."""
    csrc = os.path.join(ROOT, "clear-vae_amd", "csrc")
    r = subprocess.run(["make", "-C", csrc, "asan", "-j8"], capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-3000:]
    exe = os.path.join(ROOT, "build", "asan", "abi_asan")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0:exitcode=23")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-3000:])
    assert "AddressSanitizer" not in r.stderr
    assert "all host validation checks passed" in r.stdout
