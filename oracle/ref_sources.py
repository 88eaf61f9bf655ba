"""AST fingerprints of the reference functions the golden fixtures were generated from (build
container only; TEST INFRASTRUCTURE, see oracle/__init__). Nothing here executes reference code:
each file is parsed with ``ast`` and the named top-level definitions are hashed (``ast.dump``
without line / column attributes, so whitespace and comments do not count).

    python oracle/ref_sources.py      # writes tests/golden/reference_sources.json

``tests/test_oracle.py::test_reference_sources_unchanged`` recomputes the hashes when
/root/reference is present: a fixture generated from reference code that has since changed
fails loudly instead of pinning the oracle to stale text.
"""
import ast
import hashlib
import json
import os

REF = "/root/reference/code"
HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(os.path.dirname(HERE), "tests", "golden", "reference_sources.json")

# fixture → (reference file relative to code/, top-level definitions it was generated from)
SOURCES = {
    "objective_golden.npz": [("attack/interpolation.py", ["optimize_vgg"])],
    "patch_golden.npz": [("attack/patch/adversarial_patch.py", ["attack"]),
                         ("attack/attack_main2.py", ["patch_white_box"])],
    "fusion_golden.npz": [("attack/interpolation.py",
                           ["interpolation", "partial_adv_fusion_arithmetic"])],
    "vgg_golden.npz": [("vgg.py", ["VGGBase"])],
}


def fingerprint(path, name):
    """sha256 of the AST of the top-level def / class ``name`` in ``path`` (parsed, not run)."""
    tree = ast.parse(open(path).read())
    nodes = [n for n in tree.body
             if isinstance(n, (ast.FunctionDef, ast.ClassDef)) and n.name == name]
    if len(nodes) != 1:
        raise LookupError(f"{name}: {len(nodes)} top-level definitions in {path}")
    return hashlib.sha256(ast.dump(nodes[0], include_attributes=False).encode()).hexdigest()


def compute(ref=REF):
    return {fx: {f"{rel}::{nm}": fingerprint(os.path.join(ref, rel), nm)
                 for rel, names in entries for nm in names}
            for fx, entries in SOURCES.items()}


if __name__ == "__main__":
    with open(OUT, "w") as fh:
        json.dump(compute(), fh, indent=1, sort_keys=True)
    print("wrote", OUT)
