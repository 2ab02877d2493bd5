"""The C ABI boundary: include/dorknet_hip.h <-> libdorknet_hip.so (no GPU needed).
Loads the library, checks every declared entry point is exported with the declared
arity, and exercises the pure host-side workspace queries."""
import ctypes
import os
import re
import subprocess

import pytest

from dorknet_amd import _hip

LIB = _hip.LIB_PATH


def exported_symbols():
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], stdout=subprocess.PIPE, text=True, check=True).stdout
    return {l.split()[-1] for l in out.splitlines() if " T " in l}


def test_header_parses_and_is_complete():
    decls = _hip.parse_header()
    assert len(decls) >= 50
    for name, (ret, params) in decls.items():
        assert name.startswith("dk_") and ret in ("int", "size_t")
        for ctype, _ in params:
            _hip._argtype(ctype)  # every C type maps to a ctypes type


@pytest.mark.skipif(not os.path.exists(LIB), reason="run __graft_entry__.build() first")
def test_library_exports_exactly_the_header():
    decls = set(_hip.parse_header())
    exported = {s for s in exported_symbols() if s.startswith("dk_")}
    assert decls == exported, (decls - exported, exported - decls)


@pytest.mark.skipif(not os.path.exists(LIB), reason="run __graft_entry__.build() first")
def test_library_loads_and_host_queries_work():
    lib = _hip.lib
    assert lib.dk_abi_version() == 1
    # workspace queries are pure host functions
    assert lib.dk_conv2d_wgrad_workspace_bytes(256, 56, 56, 64, 64, 3, 3) > 0
    assert lib.dk_pwconv_wgrad_workspace_bytes(256, 56, 56, 64, 64) > 0
    assert lib.dk_dwconv_wgrad_workspace_bytes(256, 56, 56, 64, 3, 3) > 0
    assert lib.dk_dense_wgrad_workspace_bytes(256, 512, 120) > 0
    assert lib.dk_conv2d_dgrad_phase_workspace_bytes(6, 3, 5, 5, 2) == 3 * 5 * 5 * 8 * 4  # K padded to 8
    nblk = lib.dk_bn_partial_blocks(802816, 64)
    assert 1 <= nblk <= 1024
    assert lib.dk_bn_workspace_bytes(802816, 64) == nblk * 2 * 64 * 8
    fold = lib.dk_bn_partials_workspace_bytes(nblk, 64)   # the fold rows of the fixed-order reduction
    assert fold == -(-nblk // 256) * 2 * 64 * 8
    assert lib.dk_bn_bwd_workspace_bytes(802816, 64) == nblk * 2 * 64 * 8 + 2 * 64 * 4 + fold
    assert lib.dk_bn_stats_workspace_bytes(802816, 64) == nblk * 2 * 64 * 8 + fold
    assert lib.dk_colsum_workspace_bytes(1000, 10) >= 8 * 10
    assert lib.dk_l2_multi_workspace_bytes(100) == 800
    # argument errors are reported without touching the device
    with pytest.raises(_hip.HipError):
        lib.dk_conv2d_fwd_f32(0, 1, 4, 4, 3, 0, 8, 3, 3, 1, 1, 0, 0, 4, 4, None)  # C % 4 != 0
    with pytest.raises(_hip.HipError):
        lib.dk_pwconv_wgrad_f32(16, 16, 1, 4, 4, 8, 8, 1, 4, 4, 0, 0.0, 16, 16, 0, None)  # workspace too small


def test_header_matches_kernel_sources():
    """Every DK_API definition in the .hip sources is declared in the header (the sources
    #include the header, so a mismatched signature is also a compile error)."""
    csrc = os.path.join(os.path.dirname(_hip.__file__), "csrc")
    defined = set()
    for f in os.listdir(csrc):
        if f.endswith(".hip"):
            defined |= set(re.findall(r"DK_API\s+\w+\s+(dk_\w+)\s*\(", open(os.path.join(csrc, f)).read()))
    assert defined == set(_hip.parse_header())
