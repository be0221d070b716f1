"""Import this package under the name ``ldmseg_mi355x`` next to the reference's own ``ldmseg``.

The drop-in modules live in the sibling ``ldmseg/`` directory (same package name as the
reference, so the reference's tests and call sites read unchanged).  A reference checkout
that keeps its own ``ldmseg`` package (trainers, datasets, utils) binds the MI355X modules
through this alias instead — see INTEGRATION.md:

    import ldmseg_mi355x
    from ldmseg_mi355x.models import UNet, GeneralVAESeg
    from ldmseg_mi355x.schedulers import DDIMNoiseScheduler

All imports inside the package are relative, so loading the directory under a second name
is enough; nothing is copied.
"""
import importlib.util
import os
import sys

_PKG = os.path.join(os.path.dirname(os.path.abspath(__file__)), "ldmseg")

# Load ldmseg/ as a package named like this module and put it in sys.modules in this shim's
# place: the import system hands the caller whatever sys.modules holds once this file ran.
_spec = importlib.util.spec_from_file_location(__name__, os.path.join(_PKG, "__init__.py"),
                                               submodule_search_locations=[_PKG])
_pkg = importlib.util.module_from_spec(_spec)
sys.modules[__name__] = _pkg
_spec.loader.exec_module(_pkg)
