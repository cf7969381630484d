"""Drop-in for the reference's ``utils/relation.py`` (utils/relation.py:1-106):
equalization pairs (conv_k, conv_k+1, bn) along single-consumer chains.

Host-side graph logic; it only decides which HIP CLE launches run and in what
order.
"""
from __future__ import annotations

from collections import OrderedDict

from torch.nn import AvgPool2d, BatchNorm2d, ReLU

from .quantize import QConv2d, QuantMeasure

# op nodes a relation may look through (utils/relation.py:53-55)
_PASS_MODULES = (BatchNorm2d, ReLU, QuantMeasure, AvgPool2d)
_PASS_OPS = ("F.pad", "torch.mean")


class Relation:
    """(layer_first, layer_second, bn_idx) plus the accumulated scale S."""

    def __init__(self, layer_idx_1, layer_idx_2, bn_idx_1):
        self.layer_first = layer_idx_1
        self.layer_second = layer_idx_2
        self.bn_idx = bn_idx_1
        self._S = None
        self._S_lazy = None   # (flat, start, end): S as a slice of one allocation, made on first read

    @property
    def S(self):
        """The accumulated scale (a tensor, or None).  The device CLE loop hands
        every new S out as a slice of one allocation; the view object is created on
        first access (the loop itself only needs the address), which keeps ~37 view
        creations off MobileNetV2's CLE stage."""
        if self._S is None and self._S_lazy is not None:
            flat, a, b = self._S_lazy
            self._S = flat[a:b]
            self._S_lazy = None
        return self._S

    @S.setter
    def S(self, value):
        self._S = value
        self._S_lazy = None

    def _has_S(self) -> bool:
        return self._S is not None or self._S_lazy is not None

    def _set_S_lazy(self, flat, start, end):
        self._S = None
        self._S_lazy = (flat, start, end)

    def __repr__(self):
        return "({}, {})".format(self.layer_first, self.layer_second)

    def get_idxs(self):
        return self.layer_first, self.layer_second, self.bn_idx

    def set_scale_vec(self, S):
        if self.S is None:
            self.S = S
        else:
            self.S *= S

    def get_scale_vec(self):
        return self.S


def _consumer_counts(graph, bottoms):
    counts = {}
    for key in graph:
        if key == "Data":
            continue
        for b in bottoms[key]:
            counts[b] = counts.get(b, 0) + 1
    return counts


def _walk_back(graph, bottoms, start, targ_type, counts):
    """From ``start`` follow single-input, single-consumer edges upward through
    BN/ReLU/QuantMeasure/AvgPool2d and F.pad/torch.mean op nodes until a target
    layer (returned with the last BN seen) or anything else (None, None)."""
    bot = bottoms[start]
    last_bn = None
    while len(bot) == 1 and bot[0] != "Data" and counts[bot[0]] == 1:
        node = graph[bot[0]]
        if type(node) == BatchNorm2d:
            last_bn = bot[0]
        if type(node) in targ_type:
            return bot[0], last_bn
        passable = type(node) in _PASS_MODULES or (type(node) == str and any(op in bot[0] for op in _PASS_OPS))
        if not passable:
            return None, None
        bot = bottoms[bot[0]]
    return None, None


def create_relation(graph, bottoms, targ_type=[QConv2d], delete_single=False):
    """utils/relation.py:36-106.  A layer that would start two relations starts
    none (the dict pop at :76-77)."""
    counts = _consumer_counts(graph, bottoms)
    rels = OrderedDict()
    for key in graph:
        if type(graph[key]) not in targ_type:
            continue
        prev, bn = _walk_back(graph, bottoms, key, targ_type, counts)
        if prev in rels:
            rels.pop(prev)
        elif prev is not None:
            rels[prev] = Relation(prev, key, bn)
    rel_list = list(rels.values())
    if not delete_single:
        return rel_list
    # keep only chains with >= 3 target layers (relations that link up)
    groups = []
    for r in rel_list:
        home = -1
        for gi, grp in enumerate(groups):   # the last matching group wins (:87-92)
            if any(r.get_idxs()[0] == q.get_idxs()[1] for q in grp):
                home = gi
        if home >= 0:
            groups[home].append(r)
        else:
            groups.append([r])
    return [r for grp in groups if len(grp) > 1 for r in grp]
