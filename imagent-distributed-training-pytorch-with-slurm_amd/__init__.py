"""MI355X-native ImageNet data-parallel training framework.

A from-scratch re-design of the capabilities of the reference single-script
Slurm + DDP ImageNet trainer (`/root/reference/imagenet.py`) for AMD Instinct
MI355X (gfx950 / CDNA4):

* ``parallel``  - Slurm / torchrun / single-process discovery, process-group
  bootstrap, native RCCL communicator, bucketed gradient reducer, sampler.
* ``ops``       - hand-written HIP kernels (MFMA implicit-GEMM conv fwd/dgrad/
  wgrad, fused BatchNorm(+add)(+ReLU), pooling, softmax-xent+top-k, fused SGD,
  input normalisation) behind autograd Functions, with plain-PyTorch reference
  implementations used as the numerical oracle and on CPU.
* ``models``    - the ResNet family with torchvision-identical parameter names.
* ``data``      - synthetic and ImageFolder/ImageNet sources, uint8 pinned
  prefetcher with a HIP copy stream.
* ``train``     - engine (train / validate / epoch driver), LR schedule,
  optimisers, meters.
* ``utils``     - TensorBoard event writer, checkpoints, logging, profiling.

The directory name is not a valid Python identifier, so the repository ships a
``imagent_amd`` symlink to it; import the package as ``imagent_amd``.
"""

__version__ = "0.1.0"
