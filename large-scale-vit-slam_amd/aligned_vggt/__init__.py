"""MI355X-native (gfx950) implementation of the aligned_vggt package of
ruppelb/Large-Scale-ViT-SLAM: same module paths, constructor kwargs, forward
signatures and state-dict names; the hot path runs as hand-written HIP
kernels behind the C ABI in include/vggt_mi355x.h."""
