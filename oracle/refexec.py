"""Run single functions of the REFERENCE's own source (build container only; TEST INFRASTRUCTURE,
see oracle/__init__): the golden generators pin the oracle to the reference's code where that code
is plain torch but sits in modules that cannot be imported here (they import stylefusion,
torchattacks, torchvision, lpips, … at the top).

``load(path, *names)`` reads the file as text, takes the named top-level ``def``s out with ``ast``
and compiles only them. ``run_namespace(sandbox, **names)`` builds the globals they execute in:
torch / F / nn, the caller's stand-ins for the un-vendored modules, and RESTRICTED builtins — no
``__import__`` (so no import statement works), no ``eval`` / ``exec`` / ``compile``, and an
``open`` that only writes text files inside ``sandbox`` (the reference functions append their
loss logs there, e.g. ``optimize_w.txt``). ``os`` is replaced by a namespace exposing
``os.path.join`` alone.

Regenerating a golden therefore still EXECUTES reference code (the extracted function bodies);
the restrictions bound what that code can reach. Only outputs are stored under tests/golden/.
"""
import ast
import builtins
import os
import types

import torch
import torch.nn as nn
import torch.nn.functional as F

_SAFE = ("abs", "all", "any", "bool", "dict", "enumerate", "float", "int", "isinstance", "len",
         "list", "max", "min", "print", "range", "reversed", "round", "set", "sorted", "str",
         "sum", "tuple", "zip", "Exception", "ValueError", "AssertionError", "RuntimeError",
         "TypeError", "IndexError", "KeyError", "NotImplementedError", "True", "False", "None")


def load(path, *names):
    """Compile the top-level functions ``names`` of ``path`` (and nothing else of the module)."""
    tree = ast.parse(open(path).read())
    fns = [n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name in names]
    found = {n.name for n in fns}
    missing = set(names) - found
    if missing:
        raise LookupError(f"{sorted(missing)} not found in {path}")
    if len(fns) != len(names):
        raise LookupError(f"duplicate definitions of {names} in {path}")
    return compile(ast.Module(body=fns, type_ignores=[]), path, "exec")


def _sandbox_open(sandbox):
    root = os.path.realpath(sandbox)

    def _open(file, mode="r", *a, **k):
        path = os.path.realpath(str(file))
        if os.path.dirname(path) != root:
            raise PermissionError(f"reference code may only open files in {root}: {file}")
        if "b" in mode or "+" in mode:
            raise PermissionError("text read / write / append only")
        return builtins.open(path, mode, *a, **k)
    return _open


def run_namespace(sandbox, **names):
    """Globals for executing extracted reference functions (see module doc)."""
    safe = {k: getattr(builtins, k) for k in _SAFE if hasattr(builtins, k)}
    safe["open"] = _sandbox_open(sandbox)
    ns = {"__builtins__": safe, "__name__": "reference_extract", "torch": torch, "F": F,
          "nn": nn, "os": types.SimpleNamespace(path=types.SimpleNamespace(join=os.path.join))}
    ns.update(names)
    return ns


def execute(path, names, sandbox, **env):
    """Extract ``names`` from ``path`` and execute them in ``run_namespace(sandbox, **env)``;
    returns the namespace (the functions are its entries)."""
    ns = run_namespace(sandbox, **env)
    exec(load(path, *names), ns)
    return ns
