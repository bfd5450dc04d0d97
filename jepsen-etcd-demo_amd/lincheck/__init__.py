"""lincheck -- MI355X linearizability checker behind Jepsen's Checker API.

Host-side mirror of the reference interface this repository replaces
(etcdemo.clj:115-119):

    from lincheck import checker, independent, model
    chk = independent.checker(
            checker.compose({"linear": checker.linearizable(
                                 {"model": model.cas_register(), "algorithm": "linear"})}))
    result = chk.check(test, history, {})

The search runs in liblincheck.so (HIP kernels for gfx950); this package only
marshals histories and shapes results.
"""

from . import _native, history, independent, model  # noqa: F401
from . import checker  # noqa: F401
