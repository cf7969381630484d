"""Parity at the bench's full size: the exact batches bench.py times (>= 2 GiB of
fp32 weights, one plan, the production grid), checked bit-exactly against the
oracle on the first, middle and last weight set, and on every weight set through
properties that need no oracle (code range, the dequant identity under the clip,
replay idempotence)."""
import numpy as np
import pytest
import torch

import bench
from oracle import oracle as O

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
CLIP = (-15.0, 15.0)

CONFIGS = [("mobilenetv2 per-ch sym INT8 + clip + E (bench)", "mobilenetv2", 8, True, True, True)] + bench.SECONDARY


@pytest.mark.parametrize("cfg", CONFIGS, ids=[c[1] + "-" + c[0].split()[1] + f"-b{c[2]}" + ("-packed" if c[6:] and c[6] else "")
                                          for c in CONFIGS])
def test_bench_batch_vs_oracle(cfg):
    from data_free_quantization_amd.sweep import SweepPlan
    _, model, bits, channel, sym, esum, *pack = cfg
    pack = bool(pack and pack[0])
    items, shapes, per_copy, copies = bench.build_batch(model, DEV, bits=bits, channel=channel, sym=sym, esum=esum,
                                                        pack=pack)
    nl = len(shapes)
    assert len(items) == nl * copies and copies * per_copy * 4 >= 2 << 30
    plan = SweepPlan(items)
    plan.execute()
    torch.cuda.synchronize()
    mode = (2 if channel else 0) + (1 if sym else 0)
    qmin, qmax = (-(1 << (bits - 1)), (1 << (bits - 1)) - 1) if sym else (0, (1 << bits) - 1)
    sample = sorted({0, copies // 2, copies - 1})
    first = {}
    for c in sample:
        for it in items[c * nl:(c + 1) * nl]:
            x = it.src.cpu().numpy()
            rows = x.shape[0] if channel else 1
            o = O.quantize(x, bits, mode, rows=rows, khw=it.khw, flags=1, clip=CLIP, want_esum=esum)
            dq = it.dst.cpu().numpy()
            assert np.array_equal(dq, o["dq"]), (c, x.shape)
            if pack:
                oc = o["codes"].reshape(-1).astype(np.uint8) & 0xF
                oc = np.append(oc, np.zeros(oc.size % 2, np.uint8))
                assert np.array_equal(it.codes.cpu().numpy(), oc[0::2] | (oc[1::2] << 4)), (c, x.shape)
            else:
                assert np.array_equal(it.codes.cpu().numpy().view(o["codes"].dtype), o["codes"]), (c, x.shape)
            assert np.array_equal(it.scale.cpu().numpy(), o["scale"]), (c, x.shape)
            if esum:
                assert np.array_equal(it.esum.cpu().numpy(), o["esum"]), (c, x.shape)
            first[id(it)] = dq
    # every weight set: codes in range, dq == clamp(code * s + zero) bit-exactly
    for it in items:
        rows = it.src.shape[0] if channel else 1
        if pack:   # nibbles back to one code per element
            cb = it.codes.to(torch.int32)
            q = torch.stack([cb & 0xF, cb >> 4], 1).view(-1)[:it.src.numel()]
            q = torch.where(q >= 8, q - 16, q) if sym else q
            q = q.view(rows, -1)
        else:
            q = it.codes.view(rows, -1)
            if bits <= 8 and not sym:
                q = q.view(torch.uint8)
        qf = q.float()
        assert float(qf.min()) >= qmin and float(qf.max()) <= qmax
        regen = (qf * it.scale.view(-1, 1) + it.zero.view(-1, 1)).clamp(*CLIP)
        assert torch.equal(regen, it.dst.view(rows, -1))
    # replay: the same plan again gives identical outputs
    plan.execute()
    torch.cuda.synchronize()
    for c in sample:
        for it in items[c * nl:(c + 1) * nl]:
            assert np.array_equal(it.dst.cpu().numpy(), first[id(it)])
    plan.destroy()
