"""Training-loop surface (savqa_amd.train, mirroring main_itp_ddp_tar_super_node.py):
one short epoch in only_obj mode and in relation mode (only_obj off, super-node batches),
per-epoch eval (main:42-142) and the checkpoint interchange (main:425-428, eval:107-116):
the saved state_dict has the model's keys, loads back with weights_only=True, and a model
restored from it (directly or through the DDP `module.` prefix) reproduces the same
eval logits bit for bit."""
import pytest
import torch

pytestmark = pytest.mark.gpu

# tiny model: d=256, 4 heads, 2 blocks, H_mil=64, 12 classes, 5 relation categories
_ARGS = ["--local_debug", "--hidden_size", "256", "--num_heads", "4", "--num_blocks", "2",
         "--hidden_size_mil", "64", "--num_classes", "12", "--num_relations", "5",
         "--maxlen_q", "16", "--maxlen_v", "10", "--topN", "3", "--decMask",
         "--with_MILNCE_loss", "--with_smooth_labeling", "--dropout_rate", "0.5",
         "--num_epochs", "1", "--steps_per_epoch", "2", "--log_steps", "1",
         "--batch_size", "4", "--q_len", "6", "--num_regions", "5", "--num_nodes_sg", "9"]


def _model(args_maxlen, only_obj):
    from savqa_amd.AttModel_x3 import AttModel
    return AttModel(None, 256, 64, 12, 16, args_maxlen, 10, 2, 4, 0.5, 0.0, 5, only_obj,
                    device="cuda", init=False)


def _eval_logits(m, only_obj):
    from savqa_amd.data import model_args, model_args_rel, synthetic_batch, \
        synthetic_relation_batch
    if only_obj:
        b = synthetic_batch(3, Nv=5, Lq=6, Ns=9, topN=3, num_classes=12, seed=77, device="cuda")
        inp = model_args(b)
    else:
        b = synthetic_relation_batch(2, Nv=5, Lq=6, topN=3, num_relations=5, num_classes=12,
                                     seed=77, device="cuda")
        inp = model_args_rel(b)
    m.eval()
    with torch.no_grad():
        out = m(*inp, decMask=True, mcb=False)
    torch.cuda.synchronize()
    return out


@pytest.mark.parametrize("only_obj", [True, False], ids=["only_obj", "relations"])
def test_train_epoch_eval_and_checkpoint_roundtrip(tmp_path, only_obj):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from savqa_amd import train
    from savqa_amd.utils import add_module_prefix, strip_module_prefix
    maxlen = 60 if only_obj else 64  # relation mode: T_syb = 5 + 4 + 20 + 6 = 35 tokens
    argv = _ARGS + ["--maxlen", str(maxlen), "--data_dir_azure", str(tmp_path),
                    "--output_dir", "out"] + (["--only_obj"] if only_obj else [])
    res = train.cli(argv)
    assert res["epoch"] == 1
    for k in ("train_loss", "val_loss"):
        assert res[k] == res[k] and abs(res[k]) < 1e4, (k, res)  # finite
    assert 0.0 <= res["accuracy"] <= 1.0
    sd = torch.load(tmp_path / "out" / "model_1.pth", map_location="cuda", weights_only=True)
    m1 = _model(maxlen, only_obj)
    assert set(sd.keys()) == set(m1.state_dict().keys())
    m1.load_state_dict(sd)
    m2 = _model(maxlen, only_obj)
    m2.load_state_dict(strip_module_prefix(add_module_prefix(sd)))
    for k, v in m1.state_dict().items():
        assert torch.equal(v, sd[k]), k
    o1, o2 = _eval_logits(m1, only_obj), _eval_logits(m2, only_obj)
    for a, b in zip(o1[:3], o2[:3]):
        assert torch.isfinite(a).all()
        assert torch.equal(a, b)
    if not only_obj:
        assert torch.is_tensor(o1[4]) and torch.isfinite(o1[4]).all()
        assert torch.equal(o1[4], o2[4])


@pytest.mark.parametrize("only_obj", [True, False], ids=["only_obj", "relations"])
def test_train_on_gqa_files(tmp_path, only_obj):
    """main's data path end to end: GQA files (oracle/gqa_fixture.py, 2048-d features)
    -> savqa_amd.gqa reader in DataLoader workers -> collate.pack -> device padding ->
    train + eval + checkpoint."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from oracle import gqa_fixture as fx
    from savqa_amd import train
    fx.write_dataset(str(tmp_path / "gqa"), n_questions=16, fea_dim=2048)
    argv = [a for a in _ARGS]
    i = argv.index("--topN")
    argv[i + 1] = "5" if only_obj else "2"  # relation loader: topN^2 words per object pair
    argv += ["--maxlen", "80", "--with_loc", "--data_dir_azure", str(tmp_path / "gqa"),
             "--output_dir", "out", "--num_workers", "2"] + (["--only_obj"] if only_obj else [])
    res = train.cli(argv)
    assert res["epoch"] == 1
    assert res["train_loss"] == res["train_loss"] and res["val_loss"] == res["val_loss"]
    assert (tmp_path / "gqa" / "out" / "model_1.pth").exists()


def test_evaluate_matches_reference_eval():
    """train.evaluate (eval(), main:42-142) against the oracle's restatement of main:103-133
    evaluated on the REFERENCE's own logits (tests/golden/full_b4.npz): the accuracy
    numerator counts argmax hits among non-zero answers only, the denominator counts every
    sample (main:127 `cnt += batch_size`), the loss meter is sample-weighted."""
    import os
    import types
    import numpy as np
    from oracle import hashfill
    from oracle import savqa_oracle as O
    from savqa_amd.AttModel_x3 import AttModel
    from savqa_amd.data import MODEL_INPUTS
    from savqa_amd.train import evaluate
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "full_b4.npz"))
    m = AttModel(None, 512, 1024, 914, 40, 450, 49, 6, 8, 0.0, 0.0, 4, True, device="cuda",
                 init=False)
    with torch.no_grad():
        for n, p in m.named_parameters():
            p.copy_(torch.from_numpy(hashfill.param_value(n, tuple(p.shape))))
    lc, lv, ls = (torch.from_numpy(g[k]).double() for k in
                  ("logits_concat", "logits_vis", "logits_syb"))
    lsm = (torch.log_softmax(lc, -1) + torch.log_softmax(lv, -1) + torch.log_softmax(ls, -1)) / 3
    top = lsm.argmax(-1)
    # batch 1: three answers the reference predicts, one zero answer (counted in cnt only);
    # batch 2: the golden answers (mostly wrong on random weights)
    a1 = top.clone()
    a1[3] = 0
    a2 = torch.from_numpy(g["answer"])
    base = {k: torch.from_numpy(g[k]).cuda() for k in MODEL_INPUTS}
    batches = [dict(base, answer=a1.cuda()), dict(base, answer=a2.cuda())]
    args = types.SimpleNamespace(only_obj=True, decMask=bool(g["decMask"]), mcb=False)
    for with_mil in (False, True):
        loss, corr, cnt = evaluate(m, batches, with_mil, 0, args)
        mil = torch.tensor(float(g["mil_nce_obj"]), dtype=torch.float64)
        ref = O.eval_epoch([O.eval_batch(lc, lv, ls, a, mil, with_milnce=with_mil)
                            for a in (a1, a2)])
        assert cnt == ref[2] == 8
        assert corr == ref[1], (corr, ref)
        assert ref[1] >= 3
        assert abs(loss - ref[0]) < 1e-4 * abs(ref[0]), (loss, ref)
