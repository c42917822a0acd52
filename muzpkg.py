"""Import shim for the product package.

The package lives in the hyphenated directory ``exploring-muzero-on-dog_amd/`` (the
repository layout the project uses), which Python cannot import by name; ``load()``
registers it as ``exploring_muzero_on_dog_amd``.
"""
import importlib.util
import os
import sys

NAME = "exploring_muzero_on_dog_amd"
PKG_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "exploring-muzero-on-dog_amd")


def load():
    if NAME in sys.modules:
        return sys.modules[NAME]
    spec = importlib.util.spec_from_file_location(NAME, os.path.join(PKG_DIR, "__init__.py"),
                                                  submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules[NAME] = mod
    spec.loader.exec_module(mod)
    return mod
