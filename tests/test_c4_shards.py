"""Config C4 (BASELINE.json configs[3]): 128 clouds end to end, sharded over 8
ranks of 16 clouds each (bench.py --gpus 8).

The 8-GPU run itself is the driver's; what a single card can check is that
every rank's shard goes through the path each rank runs correctly.  Each of
the 8 contiguous shards ``ndnet.distributed.shard(128, 8, r)`` (clouds 16 r ..
16 r + 15 = generator seeds 16 r ..) is pushed, one after the other on one
card, through the same ``PipelinedSegmentation`` bench.py builds per rank
(bench.py:184-226: the headline U pipeline; for L the ``other_distribution``
pipeline with two NDT streams), and

  * every cloud's float32 rows hash-equal the oracle's
    (tests/golden/make_fullsize.py, config C4: seeds 0..127), and
  * the shard's log-probs equal the torch fp32 composition of the same model
    on those rows within 1e-4 (``test_model.TOL``), with the predicted class
    equal wherever the reference's top two classes are further apart than 2e-4.

Reference: /root/reference/ndnet/preprocessing/ndtnet_preprocessing.py:27-49
(the per-cloud NDT loop), /root/reference/ndnet/models/ndtnet.py:218-243.
"""
import hashlib

import numpy as np
import pytest

from conftest import golden

TOL = 1e-4
WORLD = 8


def _sha(a) -> bytes:
    return hashlib.sha256(np.ascontiguousarray(a, dtype=np.float32).tobytes()).digest()


def _bench_model(dev):
    """The model bench.py times: seed 1234, non-trivial BatchNorm statistics."""
    import torch
    from ndnet.models.ndtnet import NDTNetSegmentation
    torch.manual_seed(1234)
    model = NDTNetSegmentation(3, 28, 768).to(dev).eval()
    with torch.no_grad():
        for m in model.modules():
            if isinstance(m, torch.nn.BatchNorm1d):
                m.running_mean.uniform_(-0.2, 0.2)
                m.running_var.uniform_(0.5, 1.5)
    return model


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["U", "L"])
def test_c4_rank_shards_through_the_pipeline(kind):
    import torch
    from ndnet import distributed as D
    from ndnet.pipeline import PipelinedSegmentation
    from ndnet.synthetic import make_batch
    z = golden("fullsize_rows.npz")
    total, n = int(z["batch_C4"]), int(z["points"])
    k = int(z["levels_C4"][0])
    sha = z[f"C4_{kind}_sha"]
    assert sha.shape[0] == total == 128
    dev = torch.device("cuda", 0)
    model = _bench_model(dev)
    per_rank = D.shard(total, WORLD, 0)[1]
    pipe = PipelinedSegmentation(model, k, per_rank, n, device=dev, ndt_streams=2 if kind == "L" else None)
    seen = []
    for r in range(WORLD):
        start, count = D.shard(total, WORLD, r)
        assert count == per_rank
        seen += list(range(start, start + count))
        pipe.load_resident(torch.from_numpy(make_batch(kind, count, n, seed0=start)).to(dev))
        with torch.no_grad():
            pipe.replay()              # NDT of this shard (its forward reads the previous rows)
            out = pipe.replay()        # the forward of this shard's rows
            rows = pipe.rows[(pipe.i - 2) % pipe.R][0].clone()
            out = out.clone()
            ref = model.forward_torch(rows[..., :3].contiguous(), rows[..., 3:].contiguous())
        for plan in pipe.plans:
            plan.raise_sync_failures()
            assert all(st.rc == 0 for st in plan.host_stats()), (kind, r)
        h = rows.cpu().numpy()
        for b in range(count):
            assert _sha(h[b]) == sha[start + b, 0].tobytes(), f"C4 {kind} rank {r} cloud {start + b}"
        assert out.shape == (count, k, 29)
        err = (out - ref).abs().max().item()
        assert err < TOL, f"C4 {kind} rank {r}: forward max |diff| {err}"
        top2 = ref.topk(2, dim=-1).values
        clear = (top2[..., 0] - top2[..., 1]) > 2 * TOL
        assert torch.equal(out.argmax(-1)[clear], ref.argmax(-1)[clear]), (kind, r)
    assert seen == list(range(total))
    assert not z[f"C4_{kind}_glibc_extra"].any() and not z[f"C4_{kind}_columns_extra"].any()
