"""Stage-1 single-process generator gradients with the encoders dispatched through the
torch.library ops (product) and through the pre-round-6 direct ctypes Functions
(scripts/_encoders_direct_r6.py, a copy of that file kept for this comparison): are the
gradients bit-identical, and what are n / sum |t_i| of renderer.sigmoid_beta's sum
(tests/test_gpu_train.py::_beta_term_sum)?  Debug aid; prints one line per run.

    python scripts/beta_grad_ab.py
"""
import importlib.util
import sys
from pathlib import Path

import torch

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))


def main():
    from sdfr_loader import load
    sdfr = load()
    import sdface_gan_amd.encoders as E
    spec = importlib.util.spec_from_file_location("sdface_gan_amd._encoders_direct",
                                                  REPO / "scripts" / "_encoders_direct_r6.py")
    old = importlib.util.module_from_spec(spec)
    old.__package__ = "sdface_gan_amd"
    spec.loader.exec_module(old)
    from sdface_gan_amd.training import RendererTrainer
    from tests.test_gpu_train import (_beta_term_sum, _chunk_seeded_smoothness, _ngp_grads,
                                      _ngp_stage1_opt)
    from tests.test_train_renderer import _stage1_inputs
    torch.backends.cudnn.deterministic = True
    new_g, new_s = E.grid_encode, E.sh_encode
    opt = _ngp_stage1_opt(sdfr, True)
    ins = [_stage1_inputs(sdfr, opt, r) for r in (0, 1)]
    noise = [torch.cat([ins[0][0][0], ins[1][0][0]])]
    cams = tuple(torch.cat([a, b]) for a, b in zip(ins[0][1], ins[1][1]))
    real = torch.cat([ins[0][2], ins[1][2]])
    chunks = ins[0][3] + ins[1][3]
    opt.training.batch *= 2
    _chunk_seeded_smoothness()
    _, terms = _beta_term_sum()
    res = {}
    for name in ("ops", "direct", "ops", "direct"):
        E.grid_encode, E.sh_encode = (new_g, new_s) if name == "ops" else (old.grid_encode,
                                                                          old.sh_encode)
        terms["abs"], terms["n"] = 0.0, 0
        tr = RendererTrainer(opt, "cuda:0", seed=5)
        d, g = _ngp_grads(tr, noise, cams, real, chunks)
        b = g["renderer.sigmoid_beta"]
        print(f"{name:7s} beta grad {float(b):.10e}  n {terms['n']}  sum|t| {terms['abs']:.4e}",
              flush=True)
        if name in res:
            pd, pg = res[name]
            same = [k for k in g if not torch.equal(g[k], pg[k])]
            print(f"{name:7s} run-to-run differing generator grads: {same}", flush=True)
        res[name] = (d, g)
    go, gd = res["ops"][1], res["direct"][1]
    diff = [k for k in go if not torch.equal(go[k], gd[k])]
    print("ops vs direct differing generator grads:", diff, flush=True)


if __name__ == "__main__":
    main()
