"""CPU-side checks of the C-ABI library: it is built for gfx950, loads, and
exports every function include/comap_hip.h declares (no compute calls here)."""
import os
import re
import subprocess

import pytest

from comapreduce_amd import _native as N

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(ROOT, 'include', 'comap_hip.h')).read()
    src = re.sub(r'/\*.*?\*/', '', src, flags=re.S)
    return sorted(set(re.findall(r'\b(comap_[a-z0-9_]+)\s*\(', src)))


def test_library_exists_and_loads():
    assert os.path.exists(N.LIB_PATH), 'run __graft_entry__.build() first'
    L = N.lib()
    assert L.comap_version().startswith(b'comap_hip gfx950')


def test_every_header_symbol_exported():
    L = N.lib()
    missing = [f for f in header_functions() if not hasattr(L, f)]
    assert not missing, missing
    assert set(header_functions()) == set(N.EXPORTED), set(header_functions()) ^ set(N.EXPORTED)


def test_code_object_targets_gfx950():
    out = subprocess.run(['/opt/rocm/lib/llvm/bin/llvm-readelf', '--notes', N.LIB_PATH],
                         capture_output=True, text=True)
    if out.returncode != 0:
        pytest.skip('llvm-readelf unavailable')
    # the offload bundle carries the gfx950 code object
    data = open(N.LIB_PATH, 'rb').read()
    assert b'gfx950' in data


def test_no_gpu_context_errors_cleanly():
    import torch
    if torch.cuda.is_available():
        pytest.skip('GPU present')
    with pytest.raises(N.NativeError):
        N.ctx(0)
