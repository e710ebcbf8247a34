"""Static checks of the HIP sources (CPU, no build).

1. Every 64-bit value built from ``__builtin_amdgcn_readfirstlane`` goes through ``sgpr_u64`` /
   ``sgpr_ptr`` (snpmi_internal.hpp).  The builtin returns a 32-bit *int*: a cast of it straight to
   ``uint64_t``, or a shift of it into the high word, sign-extends a low word whose bit 31 is set --
   the illegal memory access of a round-5 A/B build (a SegFlush slot address).
2. The product kernels carry no unshipped experiment variants: the decode and CRT
   translation units have no ``SNPMI_UBENCH`` blocks.
"""
import os
import re

from conftest import ROOT

CSRC = os.path.join(ROOT, "pysnptools_amd", "csrc")
HELPER = "snpmi_internal.hpp"


def _sources():
    for name in sorted(os.listdir(CSRC)):
        if name.endswith((".hip", ".hpp")):
            with open(os.path.join(CSRC, name)) as f:
                yield name, f.read()


def _statements(text):
    """Source split into ';'-terminated statements (comments dropped), so a cast that spans lines
    is still one unit."""
    text = re.sub(r"//[^\n]*", "", text)
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return [s.strip() for s in text.split(";")]


WIDE = re.compile(r"\(\s*(?:const\s+)?(?:uint64_t|int64_t|unsigned\s+long\s+long|long\s+long|size_t|uintptr_t)\s*\)"
                  r"\s*__builtin_amdgcn_readfirstlane")


def test_readfirstlane_never_widened_directly():
    bad = []
    for name, text in _sources():
        if name == HELPER:
            continue
        for st in _statements(text):
            if "__builtin_amdgcn_readfirstlane" not in st:
                continue
            # (uint64_t)readfirstlane(...) -- the sign-extending cast
            if WIDE.search(st):
                bad.append((name, st[:160]))
            # hand-rolled hi/lo assembly of an address from readfirstlane results
            if re.search(r"<<\s*32", st) or re.search(r">>\s*32", st):
                bad.append((name, st[:160]))
    assert not bad, "64-bit values from readfirstlane must use sgpr_u64 / sgpr_ptr: %s" % bad


def test_helper_widens_through_uint32():
    text = open(os.path.join(CSRC, HELPER)).read()
    body = text[text.index("uint64_t sgpr_u64("):]
    body = body[:body.index("}")]
    assert body.count("(uint32_t)__builtin_amdgcn_readfirstlane(") == 2, body


def test_checker_catches_the_round5_pattern():
    for st in ["const uint64_t wv = (uint64_t)__builtin_amdgcn_readfirstlane(x)",
               "p = ((uint64_t)__builtin_amdgcn_readfirstlane(hi) << 32) | __builtin_amdgcn_readfirstlane(lo)"]:
        assert WIDE.search(st) or re.search(r"<<\s*32", st)


def test_product_sources_hold_no_ubench_variants():
    for name in ("kernels.hip", "syrk_crt.hip", "syrk.hip", "api.hip"):
        with open(os.path.join(CSRC, name)) as f:
            assert "SNPMI_UBENCH" not in f.read(), name
