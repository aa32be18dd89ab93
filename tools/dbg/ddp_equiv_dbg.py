"""1 rank on B vs 2 ranks on B/2 (tests/test_ddp_gpu.py's equivalence run): per step and per
tensor, the exchanged gradient against the 1-rank one and against the sum of the two ranks'
local gradients as they were when their all-reduce was issued (debug aid)."""
import os
import socket
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
import torch.multiprocessing as mp

import tests.test_ddp_gpu as T

SYNC = os.environ.get("DBG_SYNC", "")


def _patch_reducer():
    import savqa_amd.ddp as D

    class Rec(D.GradReducer):
        def begin(self):
            super().begin()
            self.local = torch.full_like(self.arena.grad, float("nan")) if self.arena.grad is not None else None
            self.issued = []

        def _dense(self, lo, hi):
            if self.arena.grad is not None:
                if getattr(self, "local", None) is None:
                    self.local = torch.full_like(self.arena.grad, float("nan"))
                self.local[lo:hi].copy_(self.arena.grad[lo:hi])
                self.issued.append((lo, hi, torch.cuda.current_stream().cuda_stream))
            super()._dense(lo, hi)
    D.GradReducer = Rec
    return Rec


def _dead(a):
    out = {}
    for n in a.order:
        o, shp = a.offsets[n]
        if o >= a.n_live:
            v = a.flat[o:o + shp.numel()].double()
            out[n] = (float(v.sum()), float(v.abs().sum()))
    return out


def worker(rank, world, port, q):
    _patch_reducer()
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from savqa_amd.data import model_args
        from savqa_amd.ddp import GradReducer
        from savqa_amd.loss import smoothed_loss
        from savqa_amd.optim import Adam
        m = T._equiv_model()
        full = T._equiv_batch()
        n = 8 // world
        batch = {k: v[rank * n:(rank + 1) * n] for k, v in full.items()}
        red = GradReducer(m._arena, bucket_mb=1.0)
        m.attach_reducer(red)
        red.sparse = []
        opt = Adam(m, lr=1e-4)
        a = m._arena
        out = []
        for step in range(2):
            red.begin()
            pre = a.flat.clone()
            lc, lv, ls, mil, _ = m(*model_args(batch), decMask=True, mcb=False)
            loss, _ = smoothed_loss(lc, lv, ls, batch["answer"], mil)
            opt.zero_grad()
            if "zg" in SYNC:
                torch.cuda.synchronize()
            loss.backward()
            if "bw" in SYNC:
                torch.cuda.synchronize()
            opt.step(reducer=red)
            torch.cuda.synchronize()
            if "late" in SYNC:
                fm = T._equiv_model()
                with torch.no_grad():
                    fm._arena.flat.copy_(pre)
                flc, flv, fls, fmil, _ = fm(*model_args(batch), decMask=True, mcb=False)
                floss, _ = smoothed_loss(flc, flv, fls, batch["answer"], fmil)
                fm._arena.ensure_grads()
                floss.backward()
                torch.cuda.synchronize()
                d = (red.local[:a.n_live] - fm._arena.grad[:a.n_live]).abs()
                print(f"rank {rank} step {step} loss {float(loss):.6f} fresh {float(floss):.6f} "
                      f"logits {float((lc - flc).abs().max()):.3e} local-vs-fresh {float(d.max()):.3e}",
                      flush=True)
                del fm
            out.append((red.local[:a.n_live].cpu().clone(), a.grad[:a.n_live].cpu().clone(),
                        list(red.issued), a.flat[:a.n_live].cpu().clone(), _dead(a),
                        {k: v.cpu().clone() for k, v in batch.items()}))
        q.put((rank, T._to_numpy(out), None))
    except Exception:
        import traceback
        q.put((rank, None, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


def ref_run():
    from savqa_amd.data import model_args
    from savqa_amd.loss import smoothed_loss
    from savqa_amd.optim import Adam
    m = T._equiv_model()
    batch = T._equiv_batch()
    opt = Adam(m, lr=1e-4)
    a = m._arena
    out = []
    flats = []
    for step in range(2):
        lc, lv, ls, mil, _ = m(*model_args(batch), decMask=True, mcb=False)
        loss, _ = smoothed_loss(lc, lv, ls, batch["answer"], mil)
        opt.zero_grad()
        loss.backward()
        torch.cuda.synchronize()
        out.append(a.grad[:a.n_live].cpu().clone())
        opt.step()
        torch.cuda.synchronize()
        flats.append((a.flat[:a.n_live].cpu().clone(), _dead(a)))
    return m, out, flats


def main():
    m, ref, rflats = ref_run()
    a = m._arena
    ctx = mp.get_context("spawn")
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    q = ctx.Queue()
    procs = [ctx.Process(target=worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r, (T._to_torch(o), e)) for r, o, e in (q.get(timeout=240) for _ in procs))
    for p in procs:
        p.join(timeout=60)
    for r in (0, 1):
        if res[r][1]:
            print(res[r][1])
            return
    print("sync", SYNC)
    f0 = res[0][0][0][3]
    worst = []
    for n in a.live_names:
        o, shp = a.offsets[n]
        d = (f0[o:o + shp.numel()] - rflats[0][0][o:o + shp.numel()]).abs()
        worst.append((float(d.max()), int((d > 1e-5).sum()), n))
    worst.sort(reverse=True)
    print("params after step 0 (max diff, #>1e-5):", worst[:8])
    for n, v in res[0][0][0][4].items():
        if v != rflats[0][1][n]:
            print("dead param differs", n, v, rflats[0][1][n])
    orig = T._equiv_batch()
    for r in (0, 1):
        for st in (0, 1):
            b = res[r][0][st][5]
            for k, v in b.items():
                o = orig[k][r * 4:(r + 1) * 4].cpu()
                if not torch.equal(v, o):
                    print("batch changed", r, st, k)
    for step in range(2):
        l0, x0, iss, _, _, _ = res[0][0][step]
        l1, x1, _, _, _, _ = res[1][0][step]
        gref = ref[step]
        print(f"== step {step}: {len(iss)} dense all-reduces, nan local {int(l0.isnan().sum())}")
        for lo, hi, st in iss:
            sl = slice(lo, hi)
            names = [n for n in a.live_names if lo <= a.offsets[n][0] < hi]
            den = float(gref[sl].double().norm()) or 1.0
            e_ex = float((x0[sl].double() / 2 - gref[sl].double()).norm()) / den
            e_loc = float(((l0[sl].double() + l1[sl].double()) / 2 - gref[sl].double()).norm()) / den
            e_sum = float((x0[sl].double() - l0[sl].double() - l1[sl].double()).norm()) / (2 * den)
            if max(e_ex, e_loc, e_sum) <= 1e-4:
                continue
            nbad = getattr(main, "nbad", 0) + 1
            main.nbad = nbad
            if nbad > 4:
                continue
            dd = ((l0[sl].double() + l1[sl].double()) / 2 - gref[sl].double()).abs()
            k = lo + int(dd.argmax())
            nm = next(n for n in a.live_names if a.offsets[n][0] <= k < a.offsets[n][0] + a.offsets[n][1].numel())
            o, shp = a.offsets[nm]
            row = (k - o) // shp[-1] if len(shp) > 1 else 0
            print(f"  [{lo},{hi}) s={st % 100000} exch-ref {e_ex:.2e} localsum-ref {e_loc:.2e} "
                  f"exch-localsum {e_sum:.2e} worst {nm} row {row}: l0 {float(l0[k]):.4g} "
                  f"l1 {float(l1[k]):.4g} ref {float(gref[k]):.4g} exch {float(x0[k]):.4g}")


if __name__ == "__main__":
    main()
