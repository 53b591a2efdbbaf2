"""sys.meta_path stub finder + timm/diffusers shim registration (golden generation only)."""
import importlib.abc
import importlib.machinery
import sys
import types

STUB_ROOTS = (
    "nuplan", "cv2", "torchvision", "shapely", "pyquaternion", "PIL",
    "pytorch_lightning", "hydra", "omegaconf", "ray",
)


class _StubMeta(type):
    def __getattr__(cls, name):
        if name.startswith("__"):
            raise AttributeError(name)
        return _make_stub_class(f"{cls.__name__}.{name}")

    def __getitem__(cls, item):
        return cls

    def __iter__(cls):
        return iter(())

    def __or__(cls, other):
        return cls


def _make_stub_class(name):
    return _StubMeta(name, (object,), {
        "__init__": lambda self, *a, **k: None,
        "__call__": lambda self, *a, **k: None,
    })


class _StubModule(types.ModuleType):
    def __init__(self, name):
        super().__init__(name)
        self.__path__ = []  # behave as a package so submodules resolve

    def __getattr__(self, name):
        if name.startswith("__"):
            raise AttributeError(name)
        val = _make_stub_class(f"{self.__name__}.{name}")
        setattr(self, name, val)
        return val


class TrajectorySampling:
    """Real stand-in for nuplan's TrajectorySampling: only the fields the config reads."""

    def __init__(self, num_poses=None, time_horizon=None, interval_length=None):
        if num_poses is None:
            num_poses = int(round(time_horizon / interval_length))
        if time_horizon is None:
            time_horizon = num_poses * interval_length
        if interval_length is None:
            interval_length = time_horizon / num_poses
        self.num_poses = num_poses
        self.time_horizon = time_horizon
        self.interval_length = interval_length

    def __hash__(self):
        return hash((self.num_poses, self.time_horizon, self.interval_length))


class _Loader(importlib.abc.Loader):
    def create_module(self, spec):
        mod = _StubModule(spec.name)
        if spec.name == "nuplan.planning.simulation.trajectory.trajectory_sampling":
            mod.TrajectorySampling = TrajectorySampling
        return mod

    def exec_module(self, module):
        return None


class _Finder(importlib.abc.MetaPathFinder):
    def find_spec(self, fullname, path=None, target=None):
        if fullname.split(".")[0] in STUB_ROOTS:
            return importlib.machinery.ModuleSpec(fullname, _Loader(), is_package=True)
        return None


def install_stub_finder():
    """Install stubs + register the timm / diffusers restatements under their import names."""
    if not any(isinstance(f, _Finder) for f in sys.meta_path):
        sys.meta_path.insert(0, _Finder())
    from . import timm_shim, diffusers_shim
    sys.modules["timm"] = timm_shim
    dmod = types.ModuleType("diffusers")
    smod = types.ModuleType("diffusers.schedulers")
    smod.DDIMScheduler = diffusers_shim.DDIMScheduler
    dmod.schedulers = smod
    dmod.DDIMScheduler = diffusers_shim.DDIMScheduler
    sys.modules["diffusers"] = dmod
    sys.modules["diffusers.schedulers"] = smod
