"""The GPU tests' engine: the product library, plus the experiments build for the kernel variants
only that build runs (`make -C smoltcp_amd/csrc EXP=1` -> smoltcp_amd/libsmolcsum_exp.so).

`VariantEngine` behaves like `smoltcp_amd.engine.ChecksumEngine` over the product library.  Forcing a
variant the product library does not carry (`set_variant`) switches every later call to a second
context over the experiments build, until the variant is reset; the tool settings (shape, grid cap,
XCD order, launch split, tile size) go to both contexts.  Without the experiments build those
variants are not run: `avail()` drops them from a loop, `need()` skips a parametrized case."""
from __future__ import annotations

import os

import pytest

from smoltcp_amd import _lib
from smoltcp_amd import engine as E


class VariantMissing(Exception):
    pass


class VariantEngine:
    _BOTH = ("set_shape", "set_max_blocks", "set_xcd_remap", "set_launch_records", "set_tile")

    def __init__(self, device: int = 0):
        self.prod = E.ChecksumEngine(device)
        self.exp = E.ChecksumEngine(device, _lib.EXP_LIB_PATH) if os.path.exists(_lib.EXP_LIB_PATH) else None
        self.cur = self.prod

    def has(self, variant: int) -> bool:
        return self.prod.variant_built(variant) or (self.exp is not None and self.exp.variant_built(variant))

    def avail(self, variants):
        """The variants of `variants` this run can force (the experiments build's only if present)."""
        return [v for v in variants if self.has(v)]

    def need(self, variant: int):
        if not self.has(variant):
            pytest.skip(f"variant {variant}: experiments build (libsmolcsum_exp.so) not built")

    def set_variant(self, variant: int):
        if self.prod.variant_built(variant):
            if self.exp is not None:
                self.exp.set_variant(-1)
            self.cur = self.prod
        elif self.exp is not None and self.exp.variant_built(variant):
            self.prod.set_variant(-1)
            self.cur = self.exp
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
