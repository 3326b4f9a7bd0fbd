"""Kernel-level check of the fused prologue + R2C pass (nft_pro_r2c.hip)
against the split passes (NFT_PRO_R2C=0): one dir-carrying forward Hartley
transform on random operands, per shape / dtype / batch: the transform (rel.
error), the direction written back (bitwise) and the d.d partials.
Usage: python tools/pror2c_check.py"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def one(shape, k, dt, lib_native, variant=""):
    _native = lib_native
    n0, n1 = shape
    P = n0 * n1
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(3)
    size = P + 64
    nf = (n0 // 2 + 1) * (n1 // 2 + 1)
    B = 777
    idx = torch.randint(0, B, (nf,), dtype=torch.int32, device=dev, generator=g)
    A = torch.randn(P, dtype=dt, device=dev, generator=g)
    XI = torch.randn(P, dtype=dt, device=dev, generator=g)
    X0 = torch.randn((k, size), dtype=dt, device=dev, generator=g)
    R = torch.randn((k, size), dtype=dt, device=dev, generator=g)
    C = torch.randn((B, k), dtype=dt, device=dev, generator=g)
    if "noc" in variant:
        C.zero_()
        XI.zero_()
    if "a1" in variant:
        A.fill_(1.0)
    SC = torch.zeros((k, _native.CG_NSCALARS), dtype=torch.float64, device=dev)
    SC[:, _native.CG_GAMMA] = 2.0
    SC[:, _native.CG_GPREV] = 1.5
    nblk = _native.hartley_dir_blocks((n0, n1))
    res = {}
    for fused in (MODE, "0"):
        os.environ["NFT_PRO_R2C"] = fused
        X = X0.clone()
        part = torch.zeros((k, nblk + 8), dtype=torch.float64, device=dev)
        s = torch.zeros((k, n0, n1), dtype=dt, device=dev)
        pro = dict(a=A.view(n0, n1), x=X[0, :], b=XI.view(n0, n1), c=C, index=idx, fold=True,
                   dir=dict(r=R[0, :], sc=SC, part=part, pstride=part.stride(0), shift=1.0, blk0=0))
        with _native.LaunchProfile() as prof:
            _native.hartley_fused(s, (1, 2), 1.0, pro=pro, convention=0, shape=s.shape,
                                  batch=dict(period=P, x=size, c=1, c_elem=k))
        if "ws" in variant:
            print("   launches:", [lab for lab, _ in prof.records])
        torch.cuda.synchronize()
        res[fused] = (s.clone(), X.clone(), part.clone())
        if "ws" in variant:
            nbytes = ctypes.c_size_t(0)
            sh = (ctypes.c_int64 * 3)(k, n0, n1)
            axx = (ctypes.c_int * 2)(1, 2)
            lib = _native.load()
            lib.nft_hartley_fused_workspace(3, sh, 2, axx, 0 if dt == torch.float64 else 1, ctypes.byref(nbytes))
            ws = _native.workspace(nbytes.value, s.device, "hartley")
            cdt = torch.complex128 if dt == torch.float64 else torch.complex64
            hs_ = (n1 // 2 + 1 + 7) // 8 * 8
            hw = ws[:k * n0 * hs_ * (16 if dt == torch.float64 else 8)].view(cdt).view(k, n0, hs_)[:, :, :n1 // 2 + 1]
            u = X[:, :P].view(k, n0, n1)
            ref = torch.fft.rfft(u, dim=-1)
            e = float(torch.linalg.vector_norm(hw - ref) / torch.linalg.vector_norm(ref))
            rowerr = (hw - ref).abs().amax(dim=-1)[0]
            bad = torch.nonzero(rowerr > 1e-6 * ref.abs().max()).flatten()[:20].tolist()
            for rr in (1, 2, 3, 255, 256, 257, 511):
                d = (hw[0, rr][None, :] - ref[0]).abs().amax(dim=-1)
                dc = (hw[0, rr][None, :] - ref[0].conj()).abs().amax(dim=-1)
                print(f"      ws row {rr}: best rfft row {int(d.argmin())} ({float(d.min()):.2e}), conj {int(dc.argmin())} ({float(dc.min()):.2e}), |row| {float(hw[0, rr].abs().max()):.2e}")
            hb = nbytes.value - 2 * k * P * (8 if dt == torch.float64 else 4)
            usp = ws[hb:hb + k * P * (8 if dt == torch.float64 else 4)].view(dt).view(k, n0, n1)
            eu = float(torch.linalg.vector_norm(usp - u) / torch.linalg.vector_norm(u))
            print(f"      u buffer vs X: {eu:.3e} (hb {hb})")
            for nm, cand in (("X0", X0), ("R", R), ("X0+R", X0 + R)):
                rc = torch.fft.rfft(cand[:, :P].view(k, n0, n1), dim=-1)
                ec = float(torch.linalg.vector_norm(hw - rc) / torch.linalg.vector_norm(rc))
                print(f"      ws vs rfft({nm}) {ec:.3e}")
            ref2 = torch.fft.fft(ref, dim=1)
            e2 = float(torch.linalg.vector_norm(hw - ref2) / torch.linalg.vector_norm(ref2))
            ratio = (hw[0, 1] / ref[0, 1])
            print(f"      ws vs colfft(rfft(u)) {e2:.3e}; ratio row1 mean {complex(ratio.mean()):.3f} std {float(ratio.abs().std()):.3f}")
            F = torch.fft.fft2(u)
            H = F.real + F.imag
            eh = float(torch.linalg.vector_norm(s - H) / torch.linalg.vector_norm(H))
            Hc = F.real - F.imag
            ehc = float(torch.linalg.vector_norm(s - Hc) / torch.linalg.vector_norm(Hc))
            print(f"   fused={fused}: ws vs rfft(u) rel {e:.3e}; bad rows {bad}; out vs Re+Im fft2(u) {eh:.3e}, Re-Im {ehc:.3e}", flush=True)
    sf, xf, pf = res[MODE]
    ss, xs, ps = res["0"]
    err = float(torch.linalg.vector_norm(sf - ss) / torch.linalg.vector_norm(ss))
    dx = bool(torch.equal(xf, xs))
    dp = float((pf - ps).abs().max() / ps.abs().max())
    print(f"{variant} {shape} k={k} {dt}: transform rel err {err:.3e}, d bitwise {dx}, partials max rel {dp:.3e}", flush=True)
    return err, dx, dp


MODE = os.environ.get("CHECK_MODE", "2")


def main():
    import nifty_amd as ift
    from nifty_amd import _native
    ift.config.set_device("cuda:0")
    bad = 0
    for shape in ((512, 512), (256, 1024), (1024, 512), (2048, 2048), (4096, 4096)):
        for dt in (torch.float64, torch.float32):
            for k in (1, 4):
                err, dx, dp = one(shape, k, dt, _native)
                tol = 1e-13 if dt == torch.float64 else 1e-5
                if not (err < tol and dx and dp < tol):
                    bad += 1
    print("BAD" if bad else "OK", bad)


if __name__ == "__main__":
    main()
