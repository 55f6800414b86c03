"""Import alias: ``import pcms_amd`` loads the package that lives in the directory
``prostate-cancer-multimodal-segmentation_amd/`` (a name Python cannot import directly).

After ``import pcms_amd`` the reference-shaped modules are available as
``pcms_amd.models.unet3d``, ``pcms_amd.utils.losses`` and ``pcms_amd.utils.trainer``.
"""
import importlib.util as _ilu
import os as _os
import sys as _sys

_PKG_DIR = _os.path.join(_os.path.dirname(_os.path.abspath(__file__)),
                         "prostate-cancer-multimodal-segmentation_amd")
_spec = _ilu.spec_from_file_location("pcms_amd", _os.path.join(_PKG_DIR, "__init__.py"),
                                     submodule_search_locations=[_PKG_DIR])
_pkg = _ilu.module_from_spec(_spec)
_sys.modules["pcms_amd"] = _pkg
_spec.loader.exec_module(_pkg)
