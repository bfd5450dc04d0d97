"""Mirror of knossos.model for this path: (model/cas-register) at etcdemo.clj:117.

Only the cas-register is implemented; the device search
takes its transition descriptors (include/lincheck.h LC_T_*).
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import Optional


@dataclass(frozen=True)
class CASRegister:
    """knossos.model/cas-register: nil initial value unless given."""
    value: Optional[int] = None

    def step(self, f: str, v):
        """Sequential spec, as knossos.model's CASRegister step (for docs/tests)."""
        if f == "write":
            return CASRegister(v)
        if f == "cas":
            cur, new = v
            if cur == self.value:
                return CASRegister(new)
            return Inconsistent(f"can't CAS {fmt(self.value)} from {fmt(cur)} to {fmt(new)}")
        if f == "read":
            if v is None or v == self.value:
                return self
            return Inconsistent(f"can't read {fmt(v)} from register {fmt(self.value)}")
        raise ValueError(f"cas-register cannot step {f!r}")


@dataclass(frozen=True)
class Inconsistent:
    msg: str


def fmt(v) -> str:
    return "nil" if v is None else str(v)


def cas_register(value: Optional[int] = None) -> CASRegister:
    if value is not None:
        raise NotImplementedError("only the nil initial value of (model/cas-register) is supported")
    return CASRegister(value)
