"""Synthetic inputs for the matchers: vocabulary, KeyFrames, MapPoints.

The reference's vocabulary file (ORBvoc) and datasets are absent offline (.MISSING_LARGE_BLOBS), so
SearchForTriangulation runs on FeatureVectors from a seeded synthetic vocabulary tree (k = 10,
2 levels, random 32-byte centroids; descent exactly as TemplatedVocabulary::transform,
TemplatedVocabulary.h:1231-1272), and SearchByProjection on seeded MapPoints built around real
extracted keypoints.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional, Tuple

import numpy as np

from . import _lib as L
from .frames import FeatureVector, Frame, LastFrameMapPoints, LocalMapPoints

_POP8 = np.array([bin(i).count("1") for i in range(256)], np.uint8)

# KITTI-like intrinsics (labelled synthetic) and arducam.yaml (TUM-shaped config)
KITTI_CAM = dict(fx=718.856, fy=718.856, cx=607.19, cy=185.22, bf=386.1448)
ARDUCAM_CAM = dict(fx=590.08, fy=590.08, cx=317.98, cy=241.15, bf=47.21)


def hamming_matrix(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """popcount(a_i xor b_j) for (n, 32) x (m, 32) uint8."""
    x = np.bitwise_xor(a[:, None, :], b[None, :, :])
    return _POP8[x].sum(axis=2, dtype=np.int32)


@dataclass
class Vocabulary:
    """A DBoW2 vocabulary tree: nodes in BFS order, children contiguous, node 0 = root.

    The reference's node table (TemplatedVocabulary::m_nodes) is `parent` / `is_leaf` /
    `descriptors` / `weights` (WordValue = double; internal nodes carry weight 0, words their idf)."""

    k: int
    levels: int
    descriptors: np.ndarray   # (n_nodes, 32) uint8 (row 0 unused: root)
    first_child: np.ndarray   # int32, -1 for leaves
    n_children: np.ndarray    # int32
    weights: np.ndarray       # float64 weight per node (word weight at the leaves)
    scoring: int = 0          # L1_NORM (ORBvoc)
    weighting: int = 0        # TF_IDF (ORBvoc)

    @property
    def n_nodes(self) -> int:
        return len(self.descriptors)

    @property
    def parent(self) -> np.ndarray:
        p = np.full(self.n_nodes, -1, np.int32)
        for node in np.nonzero(self.n_children > 0)[0]:
            p[self.first_child[node]:self.first_child[node] + self.n_children[node]] = node
        return p

    @property
    def is_leaf(self) -> np.ndarray:
        leaf = (self.n_children == 0).astype(np.uint8)
        leaf[0] = 0
        return leaf

    @staticmethod
    def synthetic(k: int = 10, levels: int = 2, seed: int = 0x0B0C0AB) -> "Vocabulary":
        rng = np.random.default_rng(seed)
        n_nodes = sum(k ** d for d in range(levels + 1))
        desc = rng.integers(0, 256, (n_nodes, 32), dtype=np.uint8)
        desc[0] = 0
        first = np.full(n_nodes, -1, np.int32)
        nch = np.zeros(n_nodes, np.int32)
        nxt = 1
        for node in range(n_nodes):
            depth = 0
            start, width = 0, 1
            while not (start <= node < start + width):
                start += width
                width *= k
                depth += 1
            if depth < levels:
                first[node] = nxt
                nch[node] = k
                nxt += k
        return Vocabulary(k, levels, desc, first, nch, np.ones(n_nodes, np.float64))

    @staticmethod
    def synthetic_orbvoc(k: int = 10, levels: int = 6, seed: int = 0x0B0C6, stop_frac: float = 0.01,
                         scoring: int = 0, weighting: int = 0) -> "Vocabulary":
        """A tree shaped like ORBvoc (k = 10, L = 6: 1,111,111 nodes, 10^6 words). Centroids are
        hierarchical -- a child differs from its parent in about 256 / 2^level bits -- so the
        descent follows real nearest-centroid paths; word weights are idf-like doubles in
        [0.5, 10), `stop_frac` of the words stopped (weight 0), internal nodes 0 (DBoW2 weights
        words only)."""
        rng = np.random.default_rng(seed)
        counts = [k ** d for d in range(levels + 1)]
        n_nodes = sum(counts)
        desc = np.zeros((n_nodes, 32), np.uint8)
        first = np.full(n_nodes, -1, np.int32)
        nch = np.zeros(n_nodes, np.int32)
        start = 1
        desc[0] = 0
        prev = slice(0, 1)
        for d in range(1, levels + 1):
            n = counts[d]
            par = np.repeat(np.arange(prev.start, prev.stop), k)
            first[prev] = start + np.arange(prev.stop - prev.start, dtype=np.int64) * k
            nch[prev] = k
            mask = rng.integers(0, 256, (n, 32), dtype=np.uint8)
            for _ in range(min(d, 5) - 1):  # P(bit flips) = 2^-min(d,5)
                mask &= rng.integers(0, 256, (n, 32), dtype=np.uint8)
            desc[start:start + n] = desc[par] ^ mask
            prev = slice(start, start + n)
            start += n
        w = np.zeros(n_nodes, np.float64)
        leaves = np.arange(prev.start, prev.stop)
        w[leaves] = rng.uniform(0.5, 10.0, len(leaves))
        w[leaves[rng.random(len(leaves)) < stop_frac]] = 0.0
        return Vocabulary(k, levels, desc, first, nch, w, scoring, weighting)

    def node_at_level(self, desc: np.ndarray, levelsup: int) -> np.ndarray:
        """TemplatedVocabulary::transform's nid for every descriptor (strict '<': first best)."""
        return self.descend(desc, levelsup)[0]

    def descend(self, desc: np.ndarray, levelsup: int) -> Tuple[np.ndarray, np.ndarray]:
        """(nid, final node) of TemplatedVocabulary::transform for every descriptor
        (TemplatedVocabulary.h:1231-1272; complete trees only)."""
        nid_level = self.levels - levelsup
        cur = np.zeros(len(desc), np.int64)
        nid = np.zeros(len(desc), np.int64)
        for level in range(1, self.levels + 1):
            best = np.full(len(desc), -1, np.int64)
            best_d = np.full(len(desc), 1 << 30, np.int64)
            for c in range(self.k):
                child = self.first_child[cur] + c
                d = _POP8[np.bitwise_xor(desc, self.descriptors[child])].sum(axis=1)
                better = d < best_d
                best_d = np.where(better, d, best_d)
                best = np.where(better, child, best)
            cur = best
            if level == nid_level:
                nid = cur.copy()
        return nid, cur

    def feature_vector(self, desc: np.ndarray, levelsup: int) -> FeatureVector:
        return FeatureVector.from_assignment(self.node_at_level(desc, levelsup))

    # ---- the reference's file formats (TemplatedVocabulary.h:1441-1461, 1516-1537) ----
    def save_text(self, path: str) -> None:
        """saveToTextFile: "k L  scoring weighting", then per node i >= 1
        "parent isLeaf d0 .. d31  weight" with the weight in ostream's default format (%g)."""
        par, leaf = self.parent, (self.n_children == 0)
        with open(path, "w") as f:
            f.write(f"{self.k} {self.levels}  {self.scoring} {self.weighting}\n")
            for i in range(1, self.n_nodes):
                d = " ".join(str(int(x)) for x in self.descriptors[i])
                f.write(f"{par[i]} {1 if leaf[i] else 0} {d}  {self.weights[i]:g}\n")

    def save_binary(self, path: str) -> None:
        """saveToBinaryFile: nb_nodes, size_node = 41, k, L, scoring, weighting; per node i >= 1
        int32 parent, 32 descriptor bytes, float32 weight, bool isLeaf."""
        n = self.n_nodes
        rec = np.zeros(n - 1, np.dtype([("p", "<i4"), ("d", "u1", 32), ("w", "<f4"), ("l", "u1")]))
        rec["p"] = self.parent[1:]
        rec["d"] = self.descriptors[1:]
        rec["w"] = self.weights[1:].astype(np.float32)
        rec["l"] = (self.n_children[1:] == 0)
        with open(path, "wb") as f:
            f.write(np.array([n, 41, self.k, self.levels, self.scoring, self.weighting], "<u4").tobytes())
            f.write(rec.tobytes())


def skew(t: np.ndarray) -> np.ndarray:
    return np.array([[0, -t[2], t[1]], [t[2], 0, -t[0]], [-t[1], t[0], 0]], np.float64)


def compute_f12(tcw1: np.ndarray, tcw2: np.ndarray, K: np.ndarray) -> np.ndarray:
    """LocalMapping::ComputeF12 (LocalMapping.cc:545-561): K1^-T [t12]x R12 K2^-1."""
    R1, t1 = tcw1[:, :3].astype(np.float64), tcw1[:, 3].astype(np.float64)
    R2, t2 = tcw2[:, :3].astype(np.float64), tcw2[:, 3].astype(np.float64)
    R12 = R1 @ R2.T
    t12 = -R1 @ R2.T @ t2 + t1
    Kd = K.astype(np.float64)
    return (np.linalg.inv(Kd).T @ skew(t12) @ R12 @ np.linalg.inv(Kd)).astype(np.float32)


def intrinsics(cam: dict) -> np.ndarray:
    return np.array([[cam["fx"], 0, cam["cx"]], [0, cam["fy"], cam["cy"]], [0, 0, 1]], np.float32)


def pose(tx=0.0, ty=0.0, tz=0.0, yaw=0.0) -> np.ndarray:
    c, s = np.cos(yaw), np.sin(yaw)
    R = np.array([[c, 0, s], [0, 1, 0], [-s, 0, c]], np.float32)
    return np.hstack([R, np.array([[tx], [ty], [tz]], np.float32)]).astype(np.float32)


def make_frame(kps: np.ndarray, desc: np.ndarray, scale: np.ndarray, sigma2: np.ndarray,
               rows: int, cols: int, cam: dict, rng: np.random.Generator,
               stereo_frac: float = 0.5, mp_frac: float = 0.3, observed_frac: float = 0.7,
               tcw: Optional[np.ndarray] = None, u_right: Optional[np.ndarray] = None) -> Frame:
    n = len(kps)
    if u_right is None:
        disp = rng.uniform(2.0, 40.0, n).astype(np.float32)
        u_right = np.where(rng.random(n) < stereo_frac, kps["x"] - disp, -1.0).astype(np.float32)
    mp = np.zeros(n, np.uint8)
    has = rng.random(n) < mp_frac
    mp[has] = np.where(rng.random(int(has.sum())) < observed_frac, L.ORBFE_MP_OBSERVED,
                       L.ORBFE_MP_PRESENT)
    return Frame(keys_un=kps, descriptors=desc if desc is not None else np.zeros((0, 32), np.uint8),
                 u_right=u_right, mp_state=mp, scale_factors=scale, level_sigma2=sigma2,
                 min_x=0.0, max_x=float(cols), min_y=0.0, max_y=float(rows),
                 tcw=tcw, **cam)


def flip_bits(desc: np.ndarray, nflips: np.ndarray, rng: np.random.Generator) -> np.ndarray:
    out = desc.copy()
    bits = np.unpackbits(out, axis=1, bitorder="little")
    for i, k in enumerate(nflips):
        if k:
            idx = rng.choice(256, int(k), replace=False)
            bits[i, idx] ^= 1
    return np.packbits(bits, axis=1, bitorder="little")


def make_local_mappoints(F: Frame, m: int, rng: np.random.Generator, match_frac: float = 0.3,
                         max_flips: int = 40, nlevels: int = 8) -> LocalMapPoints:
    """C5-style MapPoints: uniform projections; `match_frac` of them copy a nearby
    keypoint's descriptor with up to `max_flips` random bit flips."""
    n = F.N
    px = rng.uniform(F.min_x, F.max_x, m).astype(np.float32)
    py = rng.uniform(F.min_y, F.max_y, m).astype(np.float32)
    level = rng.integers(0, nlevels, m).astype(np.int32)
    desc = rng.integers(0, 256, (m, 32), dtype=np.uint8)
    sel = np.nonzero(rng.random(m) < match_frac)[0]
    if n and len(sel):
        src = rng.integers(0, n, len(sel))
        px[sel] = F.keys_un["x"][src] + rng.normal(0, 1.5, len(sel)).astype(np.float32)
        py[sel] = F.keys_un["y"][src] + rng.normal(0, 1.5, len(sel)).astype(np.float32)
        level[sel] = np.clip(F.keys_un["octave"][src] + rng.integers(0, 2, len(sel)), 0, nlevels - 1)
        desc[sel] = flip_bits(F.descriptors[src], rng.integers(0, max_flips + 1, len(sel)), rng)
    z = rng.uniform(0.5, 8.0, m).astype(np.float32)
    pxr = (px - np.float32(F.bf) / z).astype(np.float32)
    vc = rng.uniform(0.5, 1.0, m).astype(np.float32)
    vc[rng.random(m) < 0.1] = np.float32(0.9985)
    flags = np.full(m, L.MPF_TRACK_IN_VIEW | L.MPF_OBSERVED, np.uint8)
    flags[rng.random(m) < 0.05] &= ~np.uint8(L.MPF_TRACK_IN_VIEW)
    flags[rng.random(m) < 0.03] |= np.uint8(L.MPF_BAD)
    flags[rng.random(m) < 0.1] &= ~np.uint8(L.MPF_OBSERVED)
    return LocalMapPoints(flags, px, py, pxr, level, vc, desc)


def make_local_map(C: Frame, m: int, rng: np.random.Generator, match_frac: float = 0.5,
                   max_flips: int = 30) -> "MapPointGeometry":
    """Local-map MapPoints for isInFrustum + SearchByProjection (Tracking.cc:1186-1213): most lie
    in front of C near one of its keypoints, with MapPoint::UpdateNormalAndDepth-style distance
    bounds (MapPoint.cc:376-400) around C's keypoint level; the rest fail each isInFrustum test
    (behind the camera, outside the image, outside the scale-invariance range, oblique normal)."""
    from .frames import MapPointGeometry
    K = C.N
    Rcw = C.tcw[:, :3].astype(np.float64)
    tcw = C.tcw[:, 3].astype(np.float64)
    Ow = -Rcw.T @ tcw
    src = rng.integers(0, max(K, 1), m)
    z = rng.uniform(1.0, 30.0, m)
    u = (C.keys_un["x"][src] if K else rng.uniform(C.min_x, C.max_x, m)) + rng.normal(0, 1.0, m)
    v = (C.keys_un["y"][src] if K else rng.uniform(C.min_y, C.max_y, m)) + rng.normal(0, 1.0, m)
    kind = rng.random(m)
    u[kind < 0.05] = rng.uniform(-200, -10, int((kind < 0.05).sum()))  # outside the image
    pc = np.stack([(u - C.cx) / C.fx * z, (v - C.cy) / C.fy * z, z], axis=1)
    behind = (kind >= 0.05) & (kind < 0.08)
    pc[behind] *= -1.0
    pw = (Rcw.T @ (pc - tcw).T).T
    dist = np.linalg.norm(pw - Ow, axis=1)
    oct_ = C.keys_un["octave"][src] if K else np.zeros(m, np.int32)
    sf = np.float64(C.scale_factors[1]) if len(C.scale_factors) > 1 else 1.2
    nl = len(C.scale_factors)
    maxd = dist * sf ** (oct_ + rng.uniform(-0.45, 0.45, m))
    far = (kind >= 0.08) & (kind < 0.12)
    maxd[far] = dist[far] / 1.5                 # dist > 1.2 * mfMaxDistance
    mind = maxd / np.float64(C.scale_factors[nl - 1])
    near = (kind >= 0.12) & (kind < 0.15)
    mind[near] = dist[near] * 1.5               # dist < 0.8 * mfMinDistance
    nrm = (pw - Ow) / dist[:, None]
    nrm += rng.normal(0, 0.1, nrm.shape)
    oblique = (kind >= 0.15) & (kind < 0.2)
    nrm[oblique] = -nrm[oblique]
    nrm /= np.linalg.norm(nrm, axis=1)[:, None]
    desc = rng.integers(0, 256, (m, 32), dtype=np.uint8)
    sel = np.nonzero(rng.random(m) < match_frac)[0]
    if K and len(sel):
        desc[sel] = flip_bits(C.descriptors[src[sel]], rng.integers(0, max_flips + 1, len(sel)), rng)
    flags = np.full(m, L.MPF_OBSERVED, np.uint8)
    flags[rng.random(m) < 0.05] |= np.uint8(L.MPF_BAD)
    flags[rng.random(m) < 0.1] |= np.uint8(L.MPF_SEEN)
    flags[rng.random(m) < 0.2] &= ~np.uint8(L.MPF_OBSERVED)
    flags[rng.random(m) < 0.3] |= np.uint8(L.MPF_TRACK_IN_VIEW)  # stale: isInFrustum resets it
    return MapPointGeometry(flags, pw.astype(np.float32), nrm.astype(np.float32),
                            mind.astype(np.float32), maxd.astype(np.float32), desc)


def make_lastframe(C: Frame, n: int, rng: np.random.Generator, motion: np.ndarray,
                   match_frac: float = 0.6, max_flips: int = 30) -> LastFrameMapPoints:
    """Last-frame MapPoints that re-project near current keypoints after a small motion."""
    K = C.N
    tl = pose()  # last frame at the world origin
    Rcw = C.tcw[:, :3].astype(np.float64)
    tcw = C.tcw[:, 3].astype(np.float64)
    src = rng.integers(0, max(K, 1), n)
    z = rng.uniform(2.0, 20.0, n)
    u = C.keys_un["x"][src] + rng.normal(0, 1.0, n)
    v = C.keys_un["y"][src] + rng.normal(0, 1.0, n)
    pc = np.stack([(u - C.cx) / C.fx * z, (v - C.cy) / C.fy * z, z], axis=1)
    pw = (Rcw.T @ (pc - tcw).T).T.astype(np.float32)  # world point seen at (u, v) by C
    desc = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    sel = np.nonzero(rng.random(n) < match_frac)[0]
    if K and len(sel):
        desc[sel] = flip_bits(C.descriptors[src[sel]], rng.integers(0, max_flips + 1, len(sel)), rng)
    octave = np.clip(C.keys_un["octave"][src] + rng.integers(-1, 2, n), 0, len(C.scale_factors) - 1)
    angle = (C.keys_un["angle"][src] + rng.normal(0, 3.0, n)).astype(np.float32) % np.float32(360)
    wild = rng.random(n) < 0.15
    angle[wild] = rng.uniform(0, 360, int(wild.sum())).astype(np.float32)
    flags = np.full(n, L.MPF_PRESENT | L.MPF_OBSERVED, np.uint8)
    flags[rng.random(n) < 0.1] = 0
    flags[rng.random(n) < 0.05] |= np.uint8(L.MPF_OUTLIER)
    flags[rng.random(n) < 0.2] &= ~np.uint8(L.MPF_OBSERVED)
    return LastFrameMapPoints(flags, pw, desc, octave.astype(np.int32), angle, tl)


# ---- keyframe scenes (SearchByBoW, Fuse, SearchBySim3, relocalisation / loop-closing projections) ---
@dataclass
class KeyFrameScene:
    """Two KeyFrames observing one set of world points, with the MapPoints by keypoint."""

    kf1: "KeyFrame"
    kf2: "KeyFrame"
    mps1: "MapPointGeometry"   # KF1's GetMapPointMatches() by keypoint (flags 0 = NULL)
    mps2: "MapPointGeometry"
    point_of_kp1: np.ndarray   # world point index per KF1 keypoint (-1 = clutter)
    point_of_kp2: np.ndarray
    world: np.ndarray          # (P, 3) world points
    f1: Optional[Frame] = None  # the Frames the KeyFrames were made from (Frame-typed arguments)
    f2: Optional[Frame] = None


def scale_tables(sf: float, nlevels: int) -> Tuple[np.ndarray, np.ndarray]:
    """ORBextractor's mvScaleFactor / mvLevelSigma2 (ORBextractor.cc:419-426): float products."""
    scale = np.ones(nlevels, np.float32)
    for i in range(1, nlevels):
        scale[i] = np.float32(scale[i - 1] * np.float32(sf))
    return scale, (scale * scale).astype(np.float32)


def _keypoints(x, y, octave, angle, scale) -> np.ndarray:
    k = np.zeros(len(x), L.KEYPOINT_DTYPE)
    k["x"], k["y"], k["octave"] = x, y, octave
    k["size"] = np.float32(31) * scale[octave]
    k["angle"] = np.mod(angle, 360.0)
    k["response"] = 20.0
    k["class_id"] = -1
    return k


def make_keyframe_scene(rng: np.random.Generator, rows: int = 376, cols: int = 1241,
                        cam: Optional[dict] = None, n_points: int = 1200, n_clutter: int = 500,
                        t1: Optional[np.ndarray] = None, t2: Optional[np.ndarray] = None,
                        nlevels: int = 8, sf: float = 1.2, max_flips: int = 30,
                        rot_noise: float = 4.0, wild_frac: float = 0.15, bad_frac: float = 0.05,
                        stereo_frac: float = 0.4, vocab: Optional["Vocabulary"] = None,
                        levelsup: int = 0, bounds: Optional[Tuple[float, float, float, float]] = None
                        ) -> KeyFrameScene:
    """World points in front of KF1 (pixel uniform, depth 2..30 m) re-observed by KF2 where they
    project inside its image, plus clutter keypoints. Octaves follow each point's scale-invariance
    range (MapPoint::UpdateNormalAndDepth, MapPoint.cc:376-400) up to +-1; KF2 descriptors are KF1's
    with random bit flips; angles rotate by a few degrees (some wild). `bounds` = the Frame's float
    (mnMinX, mnMaxX, mnMinY, mnMaxY) of a distorted camera (KeyFrames keep their int parts)."""
    from .frames import KeyFrame, MapPointGeometry
    cam = cam or KITTI_CAM
    t1 = pose() if t1 is None else t1
    t2 = pose(tx=-0.3, tz=0.4, yaw=0.03) if t2 is None else t2
    scale, sigma2 = scale_tables(sf, nlevels)
    mnx, mxx, mny, mxy = bounds if bounds is not None else (0.0, float(cols), 0.0, float(rows))
    fx, fy, cx, cy = cam["fx"], cam["fy"], cam["cx"], cam["cy"]
    R1, p1 = t1[:, :3].astype(np.float64), t1[:, 3].astype(np.float64)
    R2, p2 = t2[:, :3].astype(np.float64), t2[:, 3].astype(np.float64)
    O1, O2 = -R1.T @ p1, -R2.T @ p2
    P = n_points
    u1 = rng.uniform(mnx + 1, mxx - 1, P)
    v1 = rng.uniform(mny + 1, mxy - 1, P)
    z = rng.uniform(2.0, 30.0, P)
    Xc1 = np.stack([(u1 - cx) / fx * z, (v1 - cy) / fy * z, z], 1)
    Xw = (R1.T @ (Xc1 - p1).T).T
    Xc2 = (R2 @ Xw.T).T + p2
    with np.errstate(divide="ignore", invalid="ignore"):
        u2 = fx * Xc2[:, 0] / Xc2[:, 2] + cx
        v2 = fy * Xc2[:, 1] / Xc2[:, 2] + cy
    in2 = (Xc2[:, 2] > 0.1) & (u2 > mnx + 1) & (u2 < mxx - 1) & (v2 > mny + 1) & (v2 < mxy - 1)
    octave = rng.integers(0, nlevels, P)
    dist1 = np.linalg.norm(Xw - O1, axis=1)
    maxd = dist1 * np.float64(sf) ** (octave + rng.uniform(-0.4, 0.4, P))
    mind = maxd / np.float64(scale[nlevels - 1])
    nrm = (Xw - O1) / dist1[:, None] + rng.normal(0, 0.05, (P, 3))
    oblique = rng.random(P) < 0.05
    nrm[oblique] = -nrm[oblique]
    nrm /= np.linalg.norm(nrm, axis=1)[:, None]
    desc = rng.integers(0, 256, (P, 32), dtype=np.uint8)
    ang = rng.uniform(0, 360, P)

    def side(sel_pts, u, v, oct_, ang_, d_, clutter):
        idx = np.nonzero(sel_pts)[0]
        n = len(idx) + clutter
        x = np.concatenate([u[idx] + rng.normal(0, 0.7, len(idx)), rng.uniform(mnx, mxx, clutter)])
        y = np.concatenate([v[idx] + rng.normal(0, 0.7, len(idx)), rng.uniform(mny, mxy, clutter)])
        o = np.concatenate([oct_[idx], rng.integers(0, nlevels, clutter)]).astype(np.int32)
        a = np.concatenate([ang_[idx], rng.uniform(0, 360, clutter)])
        d = np.concatenate([d_[idx], rng.integers(0, 256, (clutter, 32), dtype=np.uint8)])
        pid = np.concatenate([idx, np.full(clutter, -1)]).astype(np.int64)
        perm = rng.permutation(n)
        x, y, o, a, d, pid = x[perm], y[perm], o[perm], a[perm], d[perm], pid[perm]
        x = np.clip(x, mnx, mxx - 1e-3).astype(np.float32)
        y = np.clip(y, mny, mxy - 1e-3).astype(np.float32)
        return _keypoints(x, y, o, a.astype(np.float32), scale), d, pid

    k1, d1, pid1 = side(np.ones(P, bool), u1, v1, octave, ang, desc, n_clutter)
    oct2 = np.clip(octave + rng.integers(-1, 2, P), 0, nlevels - 1)
    ang2 = ang + rng.normal(0, rot_noise, P)
    wild = rng.random(P) < wild_frac
    ang2[wild] = rng.uniform(0, 360, int(wild.sum()))
    d2src = flip_bits(desc, rng.integers(0, max_flips + 1, P), rng)
    k2, d2, pid2 = side(in2, u2, v2, oct2, ang2, d2src, n_clutter)

    def frame(k, d, pid, tcw, depth):
        n = len(k)
        disp = np.where(pid >= 0, np.float32(cam["bf"]) / np.maximum(depth[np.maximum(pid, 0)], 0.1), 10.0)
        ur = np.where(rng.random(n) < stereo_frac, k["x"] - disp, -1.0).astype(np.float32)
        mp = np.where(pid >= 0, np.where(rng.random(n) < 0.7, L.ORBFE_MP_OBSERVED, L.ORBFE_MP_PRESENT),
                      L.ORBFE_MP_NONE).astype(np.uint8)
        mp[(pid >= 0) & (rng.random(n) < bad_frac)] = L.ORBFE_MP_BAD
        F = Frame(keys_un=k, descriptors=d, u_right=ur, mp_state=mp, scale_factors=scale,
                  level_sigma2=sigma2, min_x=mnx, max_x=mxx, min_y=mny, max_y=mxy, tcw=tcw, **cam)
        if vocab is not None:
            F.feat_vec = vocab.feature_vector(d, levelsup)
        return F, KeyFrame.from_frame(F)

    f1, kf1 = frame(k1, d1, pid1, t1, z)
    f2, kf2 = frame(k2, d2, pid2, t2, np.where(in2, Xc2[:, 2], 1.0))

    def geometry(kf, pid, dsrc):
        n = kf.N
        has = pid >= 0
        j = np.maximum(pid, 0)
        flags = np.where(has, L.MPF_PRESENT, 0).astype(np.uint8)
        flags[kf.mp_state == L.ORBFE_MP_BAD] |= np.uint8(L.MPF_BAD)
        pos = np.where(has[:, None], Xw[j], 0.0).astype(np.float32)
        return MapPointGeometry(flags, pos, nrm[j].astype(np.float32), mind[j].astype(np.float32),
                                maxd[j].astype(np.float32), np.where(has[:, None], dsrc[j], kf.descriptors))

    return KeyFrameScene(kf1, kf2, geometry(kf1, pid1, desc), geometry(kf2, pid2, d2src), pid1, pid2,
                         Xw.astype(np.float32), f1, f2)


def sim3_between(t1: np.ndarray, t2: np.ndarray, s12: float = 1.0):
    """(s12, R12, t12) of S12 = T1w * T2w^-1 with the scale set to s12 (LoopClosing::ComputeSim3)."""
    R1, p1 = t1[:, :3].astype(np.float64), t1[:, 3].astype(np.float64)
    R2, p2 = t2[:, :3].astype(np.float64), t2[:, 3].astype(np.float64)
    R12 = R1 @ R2.T
    t12 = p1 - s12 * R12 @ p2
    return np.float32(s12), R12.astype(np.float32), t12.astype(np.float32)


def distinctive_sets(rng: np.random.Generator, n: int, max_obs: int = 40) -> list:
    """Per-MapPoint observation descriptors: a base descriptor with a few bit flips per
    observation, some outliers, some empty sets (ComputeDistinctiveDescriptors, MapPoint.cc:272-337)."""
    out = []
    for _ in range(n):
        k = int(rng.integers(0, max_obs + 1))
        base = rng.integers(0, 256, (1, 32), dtype=np.uint8)
        d = flip_bits(np.repeat(base, k, 0), rng.integers(0, 25, k), rng) if k else np.zeros((0, 32), np.uint8)
        if k > 2:
            out_idx = rng.random(k) < 0.2
            d[out_idx] = rng.integers(0, 256, (int(out_idx.sum()), 32), dtype=np.uint8)
        out.append(d)
    return out
