"""Drop-in `import h2o` surface backed by h2o3_amd (MI355X-native)."""
from h2o3_amd.api import *  # noqa: F401,F403
from h2o3_amd.api import H2OFrame, init  # noqa: F401
from h2o3_amd import estimators  # noqa: F401
__version__ = "3.46.0.99-amd"



def _install_module_aliases():
    """Every public module path of the reference client (h2o.estimators.gbm,
    h2o.frame, h2o.tree, h2o.transforms.preprocessing, h2o.model.metrics.
    binomial, ...) resolves to a module whose names are the h2o3_amd
    implementations (table: h2o/_modules.py), so existing imports work."""
    import importlib
    import importlib.abc
    import importlib.util
    import sys
    import types
    from ._modules import MODULES
    _STAR = {"h2o.sklearn": "h2o3_amd.sklearn", "h2o.sklearn.wrapper": "h2o3_amd.sklearn",
             "h2o.tree": "h2o3_amd.tree", "h2o.tree.tree": "h2o3_amd.tree",
             "h2o.transforms": "h2o3_amd.transforms", "h2o.explanation": "h2o3_amd.explanation",
             "h2o.information_retrieval": "h2o3_amd.information_retrieval"}
    packages = {m.rsplit(".", k)[0] for m in MODULES for k in range(1, m.count("."))}

    class _Loader(importlib.abc.Loader):
        def create_module(self, spec):
            mod = types.ModuleType(spec.name)
            if spec.name in packages:
                mod.__path__ = []
            return mod

        def exec_module(self, mod):
            star = _STAR.get(mod.__name__)
            if star:                                   # names built at import time in the reference
                src_mod = importlib.import_module(star)
                for k, v in vars(src_mod).items():
                    if not k.startswith("_"):
                        setattr(mod, k, v)
            for name, src in MODULES.get(mod.__name__, {}).items():
                mname, attr = src.split(":")
                try:
                    setattr(mod, name, getattr(importlib.import_module(mname), attr))
                except (ImportError, AttributeError):
                    pass

    class _Finder(importlib.abc.MetaPathFinder):
        def find_spec(self, fullname, path, target=None):
            if fullname in MODULES or fullname in packages or fullname in _STAR:
                return importlib.util.spec_from_loader(fullname, _Loader(), is_package=fullname in packages)
            return None

    sys.meta_path.append(_Finder())
    for real in ("h2o.estimators", "h2o.grid", "h2o.automl"):   # on-disk packages: fill in the table's names
        mod = importlib.import_module(real)
        for name, src in MODULES.get(real, {}).items():
            if not hasattr(mod, name):
                mname, attr = src.split(":")
                setattr(mod, name, getattr(importlib.import_module(mname), attr))


_install_module_aliases()
