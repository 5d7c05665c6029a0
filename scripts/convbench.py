import sys, os, torch
sys.path.insert(0, os.path.join(os.getcwd(), "large-scale-vit-slam_amd"))
from aligned_vggt import _native as N
dev = torch.device("cuda:0")
def timeit(fn, reps=10):
    fn(); torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps): fn()
    b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3
for (n, hw, ci, co) in [(16, 148, 256, 256), (16, 296, 256, 128), (16, 74, 256, 256), (16, 518, 128, 32)]:
    x = torch.randn(n * hw * hw, ci, device=dev)
    w = torch.randn(co, 9 * ci, device=dev) * 0.02
    wp = torch.zeros((co + 127) // 128 * 128, 9 * ci, device=dev); wp[:co] = w
    whi, wlo = N.split_bf16x2(wp)
    b = torch.zeros(co, device=dev)
    y = torch.empty(n * hw * hw, co, device=dev)
    fl = 2 * n * hw * hw * co * 9 * ci
    outs = {}
    for pf2 in (0, 1, 0, 1):  # A/B of the gather depth (VGGT_TUNE_CONV_PF2), same process
        N.tune(N.TUNE_CONV_PF2, pf2)
        us = timeit(lambda: N.conv2d_bf16x3(x, n, hw, hw, ci, whi, wlo, b, co, 3, 3, 1, 1, y))
        outs[pf2] = y.clone()
        print(f"conv3x3 n={n} hw={hw} ci={ci} co={co} pf2={pf2}: {us:.1f} us  alg {fl/us/1e6:.0f} TF/s  "
              f"mfma {3*fl/us/1e6:.0f} TF/s", flush=True)
    print("  pf2 == one-deep bitwise:", torch.equal(outs[0], outs[1]), flush=True)
    xs = N.split_act_bf16x2(x)
    us = timeit(lambda: N.conv2d_bf16x3_pre(xs[0], xs[1], n, hw, hw, ci, whi, wlo, b, co, 3, 3, 1, 1, y))
    print(f"conv3x3 n={n} hw={hw} ci={ci} co={co} pre-split: {us:.1f} us  alg {fl/us/1e6:.0f} TF/s  "
          f"mfma {3*fl/us/1e6:.0f} TF/s  (== register-staged: {torch.equal(y, outs[1])})", flush=True)
    us = timeit(lambda: N.split_act_bf16x2(x, True, out=xs))
    print(f"  split pass: {us:.1f} us", flush=True)
    N.tune(N.TUNE_CONV_PF2, 1)
