"""A module imported on its first attribute access.  The default CLI (python -m find_circ2_amd.cli)
never needs numpy -- its search goes through pointers into libfc2.so's own buffers -- and importing
it is most of the interpreter's start-up (~0.09 s of ~0.13 s on the GPU box); the modules the CLI
imports bind ``np = LazyModule("numpy", globals(), "np")``, and the first use replaces that name with
the module itself."""
import importlib


class LazyModule:
    __slots__ = ("_name", "_namespace", "_alias")

    def __init__(self, name: str, namespace: dict, alias: str):
        self._name, self._namespace, self._alias = name, namespace, alias

    def __getattr__(self, attr):
        mod = importlib.import_module(self._name)
        self._namespace[self._alias] = mod
        return getattr(mod, attr)
