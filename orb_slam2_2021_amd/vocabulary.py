"""ORBVocabulary on MI355X: DBoW2 vocabulary descent to FeatureVector (include/orbfe_vocab.h).

Replaces the FeatureVector half of TemplatedVocabulary::transform (TemplatedVocabulary.h:1140-1272)
that KeyFrame::ComputeBoW feeds to ORBmatcher::SearchForTriangulation.
"""
from __future__ import annotations

from ctypes import byref, c_int, c_size_t, c_void_p

import numpy as np

from . import _lib as L
from .frames import FeatureVector


class ORBVocabulary:
    def __init__(self, descriptors: np.ndarray, first_child: np.ndarray, n_children: np.ndarray,
                 weights: np.ndarray, levels: int, device: int = 0):
        self._lib = L.lib()
        self.descriptors = np.ascontiguousarray(descriptors, np.uint8).reshape(-1, 32)
        self.first_child = np.ascontiguousarray(first_child, np.int32)
        self.n_children = np.ascontiguousarray(n_children, np.int32)
        self.weights = np.ascontiguousarray(weights, np.float32)
        self.levels = int(levels)
        h = c_void_p()
        L.check(self._lib.orbfe_vocab_create(len(self.descriptors), self.levels,
                                             L.ptr(self.descriptors), L.ptr(self.first_child),
                                             L.ptr(self.n_children), L.ptr(self.weights),
                                             int(device), byref(h)), "orbfe_vocab_create")
        self._h = h

    @staticmethod
    def from_tree(tree, device: int = 0) -> "ORBVocabulary":
        """From a synthetic.Vocabulary (or anything with the same fields)."""
        return ORBVocabulary(tree.descriptors, tree.first_child, tree.n_children, tree.weights,
                             tree.levels, device)

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._lib.orbfe_vocab_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def transform(self, descriptors: np.ndarray, levelsup: int = 4) -> FeatureVector:
        d = np.ascontiguousarray(descriptors, np.uint8).reshape(-1, 32)
        n = len(d)
        ids = np.zeros(max(n, 1), np.uint32)
        offs = np.zeros(n + 1, np.int32)
        idx = np.zeros(max(n, 1), np.int32)
        nn = c_int()
        L.check(self._lib.orbfe_vocab_transform(self._h, L.ptr(d), n, int(levelsup), L.ptr(ids),
                                                L.ptr(offs), L.ptr(idx), byref(nn)), "vocab_transform")
        k = nn.value
        return FeatureVector(ids[:k], offs[:k + 1], idx[:offs[k]])

    def transform_batch_device(self, n_images: int, d_desc: int, desc_stride: int, d_counts: int,
                               levelsup: int, d_node_ids: int, d_offsets: int, d_indices: int,
                               d_n_nodes: int, cap: int, stream: int = 0) -> None:
        L.check(self._lib.orbfe_vocab_transform_batch_device(
            self._h, int(n_images), c_void_p(d_desc), c_size_t(desc_stride), c_void_p(d_counts),
            int(levelsup), c_void_p(d_node_ids), c_void_p(d_offsets), c_void_p(d_indices),
            c_void_p(d_n_nodes), int(cap), c_void_p(stream)), "vocab_transform_batch_device")
