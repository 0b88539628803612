"""The GPU tests' engine: the product library, plus the experiments build for the kernel variants
only that build runs (`make -C smoltcp_amd/csrc EXP=1` -> smoltcp_amd/libsmolcsum_exp.so).

`VariantEngine` behaves like `smoltcp_amd.engine.ChecksumEngine` over the product library.  Forcing a
variant the product library does not carry (`set_variant`) switches every later call to a second
context over the experiments build, until the variant is reset; the tool settings (shape, grid cap,
XCD order, launch split, tile size) go to both contexts.

The experiments build is required: `__graft_entry__.build()` makes it next to the product library,
and a missing or stale one (another ABI version, or a variant set that lacks a product variant) fails
the first test that forces a variant, instead of silently running fewer variants.  Only with
SMOL_ALLOW_NO_EXP=1 (a product-only checkout) are its variants dropped: `avail()` leaves them out of a
loop and `need()` skips the case.  Either way the session summary says which variant set ran
(tests/conftest.py)."""
from __future__ import annotations

import os

import pytest

from smoltcp_amd import _lib
from smoltcp_amd import engine as E


class VariantMissing(Exception):
    pass


# What the session's variant tests ran on, for the summary line (tests/conftest.py).
USAGE = {"exp_lib": None, "exp_variant_runs": 0, "skipped_variants": set()}


def _exp_problem(prod: "E.ChecksumEngine", exp: "E.ChecksumEngine | None") -> str | None:
    if exp is None:
        return f"{_lib.EXP_LIB_PATH} is missing (make -C smoltcp_amd/csrc EXP=1, or __graft_entry__.build())"
    if exp._L.smol_csum_abi_version() != prod._L.smol_csum_abi_version():
        return "the experiments build has another ABI version than the product library (stale build)"
    lost = [v for v in range(-1, 128) if prod.variant_built(v) and not exp.variant_built(v)]
    if lost:
        return f"the experiments build lacks product variants {lost} (stale build)"
    return None


class VariantEngine:
    _BOTH = ("set_shape", "set_max_blocks", "set_xcd_remap", "set_launch_records", "set_tile")

    def __init__(self, device: int = 0):
        self.prod = E.ChecksumEngine(device)
        self.exp = E.ChecksumEngine(device, _lib.EXP_LIB_PATH) if os.path.exists(_lib.EXP_LIB_PATH) else None
        self.cur = self.prod
        self.allow_missing = os.environ.get("SMOL_ALLOW_NO_EXP") == "1"
        self.problem = _exp_problem(self.prod, self.exp)
        if self.problem and self.exp is not None and not self.allow_missing:
            raise RuntimeError(self.problem)
        if self.problem:
            self.exp = None
        USAGE["exp_lib"] = _lib.EXP_LIB_PATH if self.exp is not None else None

    def has(self, variant: int) -> bool:
        return self.prod.variant_built(variant) or (self.exp is not None and self.exp.variant_built(variant))

    def _missing(self, variant: int):
        if not self.allow_missing:
            pytest.fail(f"variant {variant}: {self.problem or 'not built by either library'}")
        USAGE["skipped_variants"].add(int(variant))

    def avail(self, variants):
        """The variants of `variants` this run forces: all of them (a missing one fails the test),
        or, under SMOL_ALLOW_NO_EXP=1, the ones the loaded builds carry."""
        out = []
        for v in variants:
            if self.has(v):
                out.append(v)
            else:
                self._missing(v)
        return out

    def need(self, variant: int):
        if not self.has(variant):
            self._missing(variant)
            pytest.skip(f"variant {variant}: experiments build (libsmolcsum_exp.so) not built")

    def set_variant(self, variant: int):
        if self.prod.variant_built(variant):
            if self.exp is not None:
                self.exp.set_variant(-1)
            self.cur = self.prod
        elif self.exp is not None and self.exp.variant_built(variant):
            self.prod.set_variant(-1)
            self.cur = self.exp
            USAGE["exp_variant_runs"] += 1
        else:
            raise VariantMissing(variant)
        self.cur.set_variant(variant)

    def close(self):
        self.prod.close()
        if self.exp is not None:
            self.exp.close()

    def __getattr__(self, name):
        if name in self._BOTH:
            def both(*a, **k):
                out = getattr(self.prod, name)(*a, **k)
                if self.exp is not None:
                    getattr(self.exp, name)(*a, **k)
                return out
            return both
        return getattr(self.cur, name)
