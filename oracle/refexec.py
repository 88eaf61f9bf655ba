"""Run single functions of the REFERENCE's own source (build container only; TEST INFRASTRUCTURE,
see oracle/__init__): the golden generators pin the oracle to the reference's code where that code
is plain torch but sits in modules that cannot be imported here (they import stylefusion,
torchattacks, torchvision, lpips, … at the top).

``load(path, *names)`` reads the file as text, takes the named top-level ``def``s out with ``ast``
and compiles only them. ``run_namespace(workdir, **names)`` builds the globals they execute in:
torch / F / nn, the caller's stand-ins for the un-vendored modules, a reduced builtins table (no
``__import__``, ``eval``, ``exec``, ``compile``) and an ``open`` limited to text files directly
inside ``workdir`` (the reference functions append their loss logs there, e.g.
``optimize_w.txt``).

THIS IS NOT A SANDBOX. The namespace hands the extracted code the real ``torch`` module, and
through it ``torch.os``, ``torch.sys``, ``torch.load`` and the rest of the process: code that
wanted to could reach the file system, spawn processes or unpickle data. The reduced builtins
only keep the extracted functions from importing the rest of the reference and keep their log
files in a temporary directory; they bound nothing against hostile code. Executing reference
code is therefore an explicit, manual act: ``execute`` refuses unless ``MIA_EXEC_REFERENCE=1`` is
set, the generators run it once in the build container as a separate throwaway process
(``python oracle/gen_golden_*.py``), and nothing in tests/, bench.py or smoke() calls it. Only
outputs (arrays) are stored under tests/golden/; ``oracle/ref_sources.py`` records, WITHOUT
executing anything, an AST hash of every reference function a fixture was generated from, so a
CPU test notices when the reference text changes under a fixture.
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


def _workdir_open(workdir):
    root = os.path.realpath(workdir)

    def _open(file, mode="r", *a, **k):
        path = os.path.realpath(str(file))
        if os.path.dirname(path) != root:
            raise PermissionError(f"extracted code may only open files in {root}: {file}")
        if "b" in mode or "+" in mode:
            raise PermissionError("text read / write / append only")
        return builtins.open(path, mode, *a, **k)
    return _open


def run_namespace(workdir, **names):
    """Globals for executing extracted reference functions (see module doc: not a sandbox)."""
    safe = {k: getattr(builtins, k) for k in _SAFE if hasattr(builtins, k)}
    safe["open"] = _workdir_open(workdir)
    ns = {"__builtins__": safe, "__name__": "reference_extract", "torch": torch, "F": F,
          "nn": nn, "os": types.SimpleNamespace(path=types.SimpleNamespace(join=os.path.join))}
    ns.update(names)
    return ns


def execute(path, names, workdir, **env):
    """Extract ``names`` from ``path`` and execute them in ``run_namespace(workdir, **env)``;
    returns the namespace (the functions are its entries). Runs reference code with this
    process's full privileges: requires ``MIA_EXEC_REFERENCE=1`` (module doc)."""
    if os.environ.get("MIA_EXEC_REFERENCE") != "1":
        raise PermissionError("executing reference code is a manual golden-generation step: "
                              "set MIA_EXEC_REFERENCE=1 (this is not a sandbox; see refexec)")
    ns = run_namespace(workdir, **env)
    exec(load(path, *names), ns)
    return ns
