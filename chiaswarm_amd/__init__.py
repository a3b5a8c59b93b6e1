"""chiaswarm_amd — an MI355X-native (gfx950 / CDNA4) distributed diffusion worker.

Same hive protocol, job schema and result envelope as the chiaSWARM worker
(reference: swarm/__init__.py:1 reports worker version 0.23.6), rebuilt around
PyTorch-ROCm + hand-written HIP kernels (csrc/kernels/*.hip) + RCCL over xGMI.

``__version__`` is the *protocol* version reported to the hive as
``worker_version`` (hive-visible, kept compatible with the reference);
``__framework_version__`` is this implementation's own version.
"""

__version__ = "0.23.6"
__framework_version__ = "0.1.0"
