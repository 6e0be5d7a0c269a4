"""CPU: the C-ABI library builds, loads, and exports every symbol include/mmla.h declares.
No compute calls (there is no GPU here); creating a context without a device must fail cleanly."""
import ctypes
import os
import re

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, 'include', 'mmla.h')
LIB = os.path.join(REPO, 'mmla_audio_amd', 'libmmla.so')


def declared_symbols():
    src = open(HEADER).read()
    return sorted(set(re.findall(r'^\s*(?:int|const char\*)\s+(mmla_\w+)\s*\(', src, re.M)))


def test_header_declares_expected_entry_points():
    syms = declared_symbols()
    for s in ('mmla_create', 'mmla_destroy', 'mmla_load_weights', 'mmla_od_features',
              'mmla_si_features', 'mmla_si_features_seq', 'mmla_od_forward', 'mmla_si_forward',
              'mmla_od_pipeline', 'mmla_si_pipeline', 'mmla_last_error'):
        assert s in syms


@pytest.fixture(scope='module')
def lib():
    if not os.path.exists(LIB):
        pytest.skip('libmmla.so not built (run __graft_entry__.build())')
    return ctypes.CDLL(LIB)


def test_library_exports_every_declared_symbol(lib):
    for s in declared_symbols():
        assert hasattr(lib, s), f'{s} declared in include/mmla.h but not exported'


def test_shim_signatures_cover_header():
    from mmla_audio_amd import _lib
    declared = set(declared_symbols()) - {'mmla_last_error'}
    assert declared == set(_lib.SIGNATURES), declared ^ set(_lib.SIGNATURES)


def test_abi_version(lib):
    assert lib.mmla_abi_version() == 2


def test_null_args_rejected_without_device(lib):
    lib.mmla_create.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]
    assert lib.mmla_create(0, None) == -1          # MMLA_E_INVALID before touching HIP
    lib.mmla_destroy.argtypes = [ctypes.c_void_p]
    assert lib.mmla_destroy(None) == -1


def test_package_imports_without_gpu():
    import mmla_audio_amd
    from mmla_audio_amd import weights
    assert weights.n_params(weights.OD) > 1_000_000
    assert mmla_audio_amd.__doc__
