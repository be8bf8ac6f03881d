"""two_tower_recommender_model_amd — MI355X-native (gfx950) hot path of the two-tower training step of
alexmillerdb/two_tower_recommender_model, behind the torchrec API the reference uses.

    import two_tower_recommender_model_amd as tt
    tt.install_torchrec_alias()          # `import torchrec...` now resolves to tt.torchrec
    from torchrec.distributed import TrainPipelineSparseDist   # ... the reference loop runs as is

Kernels: libtt_mi355x.so (C ABI, include/tt_mi355x.h), loaded through ctypes by ``_lib``.
"""
from __future__ import annotations

import importlib
import importlib.abc
import importlib.util
import sys

__version__ = "0.1.0"

_ALIAS = "torchrec"
_REAL = __name__ + ".torchrec"


class _AliasFinder(importlib.abc.MetaPathFinder, importlib.abc.Loader):
    """Resolve ``torchrec[.x.y]`` to ``two_tower_recommender_model_amd.torchrec[.x.y]`` (same module
    objects, so isinstance checks agree between the two names)."""

    def find_spec(self, fullname, path=None, target=None):
        if fullname == _ALIAS or fullname.startswith(_ALIAS + "."):
            real = _REAL + fullname[len(_ALIAS):]
            if importlib.util.find_spec(real) is None:
                return None
            return importlib.util.spec_from_loader(fullname, self, is_package=True)
        return None

    def create_module(self, spec):
        real = _REAL + spec.name[len(_ALIAS):]
        return importlib.import_module(real)

    def exec_module(self, module):
        pass


def install_torchrec_alias() -> None:
    if not any(isinstance(f, _AliasFinder) for f in sys.meta_path):
        sys.meta_path.insert(0, _AliasFinder())
