"""1x1-conv weight gradients (a plain TN GEMM: dW[Co][Ci] += dY^T X over all
pixels) on the hand-written wgrad kernel vs hipBLASLt through torch.addmm
(bf16 in, fp32 accumulate into the existing gradient)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch


def timeit(fn, reps=10, warm=3):
    for _ in range(warm):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    from imagent_amd.ops.conv import igemm_wgrad
    B = 512
    shapes = [(64, 56, 64), (64, 56, 256), (256, 56, 64), (256, 56, 128), (128, 28, 512), (512, 28, 128),
              (512, 28, 256), (256, 14, 1024), (1024, 14, 256), (1024, 14, 512), (512, 7, 2048), (2048, 7, 512)]
    for Ci, H, Co in shapes:
        M = B * H * H
        x = torch.randn(B, H, H, Ci, device="cuda").to(torch.bfloat16)
        dy = torch.randn(B, H, H, Co, device="cuda").to(torch.bfloat16)
        dw = torch.zeros(Co, 1, 1, Ci, device="cuda")
        t0 = timeit(lambda: igemm_wgrad(dy, x, dw, 1, 0, 1, 1))
        a, b = dy.view(M, Co).t(), x.view(M, Ci)
        dw2 = torch.zeros(Co, Ci, device="cuda")
        try:
            t1 = timeit(lambda: torch.addmm(dw2, a, b, out_dtype=torch.float32, out=dw2))
        except Exception as e:  # noqa
            print("addmm out_dtype failed:", e)
            t1 = float("nan")
        t2 = timeit(lambda: torch.mm(a, b))
        dw.zero_()
        dw2.zero_()
        igemm_wgrad(dy, x, dw, 1, 0, 1, 1)
        try:
            torch.addmm(dw2, a, b, out_dtype=torch.float32, out=dw2)
            err = ((dw.view(Co, Ci) - dw2).norm() / dw2.norm()).item()
        except Exception:
            err = float("nan")
        fl = 2.0 * M * Co * Ci
        print(f"{Ci:5d} {H:3d} {Co:5d} | hip {t0:7.1f} us {fl / t0 / 1e6:5.0f} TF | addmm-f32 {t1:7.1f} us "
              f"{fl / t1 / 1e6:5.0f} TF | mm-bf16 {t2:7.1f} us | rel {err:.2e}", flush=True)


if __name__ == "__main__":
    main()
