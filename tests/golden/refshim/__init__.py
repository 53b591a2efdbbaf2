"""Offline import shims for the reference DiffusionDrive model (golden-vector generation ONLY).

This package lets ``tests/golden/make_golden.py`` import
``navsim.agents.diffusiondrive.transfuser_model_v2`` from ``/root/reference`` inside
the build container, where the reference's third-party dependencies are absent
(SURVEY.md §8c). Nothing here is imported by the product package, by ``bench.py``
or by any ``-m gpu`` test; ``/root/reference`` does not exist on the GPU box.

Three kinds of shim:

* ``install_stub_finder()`` — a ``sys.meta_path`` finder returning permissive stub
  modules for packages the model file imports only for type names / training code
  (nuplan, cv2, torchvision, shapely, pyquaternion, PIL, pytorch_lightning, hydra,
  omegaconf). ``nuplan...TrajectorySampling`` is real (``num_poses = horizon/interval``)
  because ``TransfuserConfig`` (transfuser_config.py:14-15) reads ``num_poses``.
* ``timm`` — restatement of timm's ResNet ``features_only`` trunk (module names,
  ``return_layers`` and ``feature_info`` as transfuser_backbone.py:24-33,50-55,62-65
  consume them). timm is unpinned (requirements.txt:49): parity is unpinned at
  this boundary, our restatement is what the goldens pin.
* ``diffusers`` — restatement of ``DDIMScheduler`` defaults as used at
  transfuser_model_v2.py:447-451,584,595-597,634-636 (unpinned, docs/install.md:7).
"""
from .stubs import install_stub_finder  # noqa: F401
