"""Import helper: registers the ``sdface-gan_amd/`` package as ``sdface_gan_amd``.

    from sdfr_loader import load
    sdfr = load()            # == import sdface_gan_amd
"""
from __future__ import annotations

import importlib.util
import sys
from pathlib import Path

PKG_NAME = "sdface_gan_amd"
PKG_DIR = Path(__file__).resolve().parent / "sdface-gan_amd"


def load():
    mod = sys.modules.get(PKG_NAME)
    if mod is not None:
        return mod
    spec = importlib.util.spec_from_file_location(
        PKG_NAME, PKG_DIR / "__init__.py", submodule_search_locations=[str(PKG_DIR)])
    mod = importlib.util.module_from_spec(spec)
    sys.modules[PKG_NAME] = mod
    try:
        spec.loader.exec_module(mod)
    except BaseException:
        del sys.modules[PKG_NAME]
        raise
    return mod
