"""MI355X-native (gfx950) implementation of the aligned_vggt package of
ruppelb/Large-Scale-ViT-SLAM: same module paths, constructor kwargs, forward
signatures and state-dict names; the hot path runs as hand-written HIP
kernels behind the C ABI in include/vggt_mi355x.h."""
import os as _os

# Kernel arguments in device memory: the command processor then does not read
# each dispatch's arguments over PCIe, which shortens the dispatch-to-dispatch
# time of dependent kernels (profiles/r6h: aggregator step -1.1 %, configs[3]
# -2.2 %, training step -4.5 %).  Read by the HIP runtime at initialisation, so
# it only takes effect when this package is imported before the first GPU call.
_os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")
# The multi-GPU ring's encode gate (runtime.EncodeGate) parks the encode stream with
# hipStreamWaitValue32.  By default the HIP runtime implements that wait as a
# polling kernel on the GPU, and while it polls every kernel of the alignment it
# gates for runs slower: align_chunk 2.61 -> 3.45-3.51 ms at the configs[3] shape.
# This flag makes the command processor wait on the value instead (an AQL
# barrier-value packet, no kernel): 2.68 -> 2.87 ms, the rest being the encode
# work still in flight (scripts/gate_probe.py, profiles/r10/gate_probe_*).  Same
# ordering semantics; read at HIP initialisation like the flag above.
_os.environ.setdefault("GPU_STREAMOPS_CP_WAIT", "1")
