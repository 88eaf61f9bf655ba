"""Import shim: exposes the package directory
``adversarial-attacks-on-gan-based-image-fusion_amd/`` (not a valid Python identifier)
as the importable package ``gfa_amd``.

    import gfa_import  # noqa: F401
    from gfa_amd import attack
"""
import importlib.util
import os
import sys

PKG_NAME = "gfa_amd"
PKG_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)),
                       "adversarial-attacks-on-gan-based-image-fusion_amd")


def load():
    if PKG_NAME in sys.modules:
        return sys.modules[PKG_NAME]
    spec = importlib.util.spec_from_file_location(
        PKG_NAME, os.path.join(PKG_DIR, "__init__.py"), submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules[PKG_NAME] = mod
    try:
        spec.loader.exec_module(mod)
    except BaseException:
        del sys.modules[PKG_NAME]
        raise
    return mod


load()
