"""CPU checks of the drop-in boundary: libmatternet_hip.so loads and exports
every symbol include/*.h declares; argument validation fails loudly without
touching the GPU (no compute calls here)."""
import ctypes as C
import glob
import os
import re

import pytest

import surfface_hip
from surfface_hip import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_symbols():
    syms = set()
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        text = open(h).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        for m in re.finditer(r"\b(mn_[a-z0-9_]+)\s*\(", text):
            syms.add(m.group(1))
    return syms


def test_library_exports_every_declared_symbol():
    L = _lib.lib()
    declared = _declared_symbols()
    assert declared, "no mn_* declarations found in include/"
    missing = [s for s in sorted(declared) if not hasattr(L, s)]
    assert not missing, missing
    # and the Python binding declares a signature for each
    assert declared <= set(_lib.SIGNATURES), declared - set(_lib.SIGNATURES)


def test_version_and_error_paths_without_gpu():
    L = _lib.lib()
    assert L.mn_version() >= 100
    # NULL opts / pointers are rejected before any HIP call
    assert L.mn_knn_f32(None, 10, 4, None, None, None) == _lib.MN_EINVAL
    assert b"opts" in L.mn_last_error()
    o = _lib.KnnOpts(k=0, metric=0, exclude_self=1, margin=0, timing=0, algo=0, stream=None)
    assert L.mn_knn_f32(C.c_void_p(16), 10, 4, C.byref(o), C.c_void_p(16), C.c_void_p(16)) \
        == _lib.MN_ENOTSUP
    o.k, o.metric = 5, 7
    assert L.mn_knn_f32(C.c_void_p(16), 10, 4, C.byref(o), C.c_void_p(16), C.c_void_p(16)) \
        == _lib.MN_ENOTSUP
    with pytest.raises(surfface_hip.MnError):
        _lib.check(_lib.MN_EINVAL)


def test_no_cpu_fallback_in_product_path():
    """The product package must not import the oracle (test infrastructure)."""
    pkg = os.path.join(ROOT, "matternet-rs_amd")
    for path in glob.glob(os.path.join(pkg, "**", "*.py"), recursive=True) + \
            glob.glob(os.path.join(pkg, "csrc", "*")):
        if os.path.isdir(path):
            continue
        text = open(path, errors="ignore").read()
        assert not re.search(r"import\s+oracle|from\s+oracle|liboracle|\bor_[a-z0-9_]+\(", text), path


def test_release_library_has_no_probes_or_tuning_knobs():
    """the release .so cannot be switched into a timing
    probe (results invalid, MN_OK) or an A/B path by a stray environment
    variable.  The probe kernel instantiations (PROBE != 0 template argument)
    and the MN_* tuning variable names exist only in the tuning build; the
    release library reads only the diagnostics MN_DEBUG_SYNC / MN_X1_DEBUG."""
    blob = open(_lib.LIB_PATH, "rb").read()
    # k_gram_sweep2<PROBE, ...> / k_gram_bf16<MODE, PROBE>: only PROBE = 0
    assert re.search(rb"k_gram_sweep2ILi0E", blob)
    assert not re.search(rb"k_gram_sweep2ILi[1-9]E", blob)
    assert re.search(rb"k_gram_sweep3ILi0E", blob) and not re.search(rb"k_gram_sweep3ILi[1-9]E", blob)
    assert not re.search(rb"k_gram_bf16ILi\d+ELi[1-9]E", blob)
    # the legacy sweep of gram_sweep.hpp is gone
    assert not re.search(rb"k_gram_sweepILi", blob)
    # MN_* names in the binary: the header's own constants (error texts) and
    # the two diagnostics only
    consts = set(re.findall(rb"\b(MN_[A-Z0-9_]+)\b",
                            open(os.path.join(ROOT, "include", "matternet_hip.h"), "rb").read()))
    names = set(re.findall(rb"MN_[A-Z0-9_]{3,}", blob)) - consts
    assert names <= {b"MN_DEBUG_SYNC", b"MN_X1_DEBUG"}, names
    # the tuning build carries them (scripts/ and alternative-path tests)
    if os.path.exists(_lib.TUNING_LIB_PATH):
        tb = open(_lib.TUNING_LIB_PATH, "rb").read()
        assert b"MN_X1_PROBE" in tb and re.search(rb"k_gram_sweep2ILi1E", tb)


def test_lexicographic_rank_formula_matches_string_sort():
    """The closed-form rank used by k_make_keys (sorted_index.hip), restated."""
    def cwp(v, N):
        c, lo, hi = 0, v, v
        while lo < N:
            c += min(hi, N - 1) - lo + 1
            lo, hi = lo * 10, hi * 10 + 9
        return c

    def lexrank(i, N):
        if i == 0:
            return 0
        s = str(i)
        r, pre = len(s), 0
        for p, ch in enumerate(s):
            for c in range(1 if p == 0 else 0, int(ch)):
                r += cwp(pre * 10 + c, N)
            pre = pre * 10 + int(ch)
        return r

    for N in (1, 2, 9, 10, 11, 100, 101, 999, 1000, 4321):
        ranks = {v: k for k, v in enumerate(sorted(range(N), key=str))}
        assert all(lexrank(i, N) == ranks[i] for i in range(N))
