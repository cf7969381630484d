"""Debug: device CLE metric vs the oracle for one relation at several sizes."""
import sys
from collections import OrderedDict
from pathlib import Path

import numpy as np
import torch
import torch.nn as nn

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from oracle import oracle as O  # noqa: E402
from data_free_quantization_amd import Cross_layer_equal as cle  # noqa: E402
from data_free_quantization_amd.utils.relation import Relation  # noqa: E402


class BN:
    pass


for (c1, l1, o2) in [(4, 2, 3), (16, 27, 8), (64, 200, 16), (128, 128, 4), (256, 600, 8), (512, 300, 1000)]:
    rng = np.random.default_rng(0)
    w1 = rng.normal(0, 1, (c1, l1)).astype(np.float32)
    w2 = rng.normal(0, 1, (o2, c1)).astype(np.float32)
    g = OrderedDict()
    g["Data"] = "Data"
    a = nn.Linear(l1, c1).cuda()
    a.weight.data = torch.from_numpy(w1).cuda()
    a.bias.data = torch.zeros(c1).cuda()
    b = nn.Linear(c1, o2).cuda()
    b.weight.data = torch.from_numpy(w2).cuda()
    bn = BN()
    bn.fake_weight = torch.ones(c1).cuda()
    bn.fake_bias = torch.zeros(c1).cuda()
    g["a"], g["bn"], g["b"] = a, bn, b
    cle.cross_layer_equalization(g, [Relation("a", "b", "bn")], [nn.Linear], Treshhold=1e3, Save_state=False)
    r1, r2, _, _, _, _ = O.cle_relation(w1, w2, np.zeros(c1, np.float32), np.ones(c1, np.float32),
                                         np.zeros(c1, np.float32))
    m1 = O.mean_abs_diff(r1, w1)
    m2 = O.mean_abs_diff(r2, w2)
    ref = O.np_sum([m1, m2])
    got = cle.LAST_RUN["diffs"][0]
    ok1 = np.array_equal(a.weight.detach().cpu().numpy(), r1)
    ok2 = np.array_equal(b.weight.detach().cpu().numpy(), r2)
    print((c1, l1, o2), "n1", c1 * l1, "n2", o2 * c1, "weights ok", ok1, ok2, "diff", got, ref, got == ref,
          "m1", m1, "m2", m2, flush=True)

