"""The device's closed-form inverse of an AnimatedPrimitive's transform
(pt_shading.h anim_inverse) against glm::inverse's general formula
(compute_inverse<4,4>) evaluated op by op in float32 with every operation
rounded -- the form the oracle's mat4_inverse_ restates (oracle/pt_oracle.c)
and the motion parity scenes pin against the reference harness: identity +
translation column v, v finite and never -0 (anim_transform adds +0), bit for
bit, zero signs included."""
import numpy as np

f32 = np.float32


def general_inverse(T):
    """compute_inverse<4,4> on arrays of column-major matrices T[..., 16]."""
    M = lambda c, r: T[..., c * 4 + r]  # noqa: E731
    D2 = lambda a, b, c, d: (a * b) - (c * d)  # noqa: E731
    C = {}
    for name, (a, b, c, d) in {
            "00": ((2, 2), (3, 3), (3, 2), (2, 3)), "02": ((1, 2), (3, 3), (3, 2), (1, 3)),
            "03": ((1, 2), (2, 3), (2, 2), (1, 3)), "04": ((2, 1), (3, 3), (3, 1), (2, 3)),
            "06": ((1, 1), (3, 3), (3, 1), (1, 3)), "07": ((1, 1), (2, 3), (2, 1), (1, 3)),
            "08": ((2, 1), (3, 2), (3, 1), (2, 2)), "10": ((1, 1), (3, 2), (3, 1), (1, 2)),
            "11": ((1, 1), (2, 2), (2, 1), (1, 2)), "12": ((2, 0), (3, 3), (3, 0), (2, 3)),
            "14": ((1, 0), (3, 3), (3, 0), (1, 3)), "15": ((1, 0), (2, 3), (2, 0), (1, 3)),
            "16": ((2, 0), (3, 2), (3, 0), (2, 2)), "18": ((1, 0), (3, 2), (3, 0), (1, 2)),
            "19": ((1, 0), (2, 2), (2, 0), (1, 2)), "20": ((2, 0), (3, 1), (3, 0), (2, 1)),
            "22": ((1, 0), (3, 1), (3, 0), (1, 1)), "23": ((1, 0), (2, 1), (2, 0), (1, 1))}.items():
        C[name] = D2(M(*a), M(*b), M(*c), M(*d))
    F = [[C["00"], C["00"], C["02"], C["03"]], [C["04"], C["04"], C["06"], C["07"]],
         [C["08"], C["08"], C["10"], C["11"]], [C["12"], C["12"], C["14"], C["15"]],
         [C["16"], C["16"], C["18"], C["19"]], [C["20"], C["20"], C["22"], C["23"]]]
    V = [[M(1, k), M(0, k), M(0, k), M(0, k)] for k in range(4)]
    comb = [(1, 0, 2, 1, 3, 2), (0, 0, 2, 3, 3, 4), (0, 1, 1, 3, 3, 5), (0, 2, 1, 4, 2, 5)]
    inv = [[None] * 4 for _ in range(4)]
    for i, c in enumerate(comb):
        sg = f32(-1.0) if i & 1 else f32(1.0)
        for k in range(4):
            v = (V[c[0]][k] * F[c[1]][k] - V[c[2]][k] * F[c[3]][k]) + V[c[4]][k] * F[c[5]][k]
            inv[i][k] = v * (-sg if k & 1 else sg)
    d0 = [M(0, k) * inv[k][0] for k in range(4)]
    od = f32(1.0) / ((d0[0] + d0[1]) + (d0[2] + d0[3]))
    return np.stack([inv[c][r] * od for c in range(4) for r in range(4)], axis=-1)


def closed_form(v):
    out = np.tile(np.array([1.0, -0.0, 0.0, -0.0, -0.0, 1.0, -0.0, 0.0, 0.0, -0.0, 1.0, -0.0, 0, 0, 0, 1.0],
                           np.float32), (len(v), 1))
    out[:, 12] = -v[:, 0]
    out[:, 13] = f32(0.0) - v[:, 1]
    out[:, 14] = -v[:, 2]
    return out


def test_translation_inverse_closed_form_matches_the_general_formula():
    rng = np.random.default_rng(7)
    vs = rng.integers(0, 2**32, size=(200_000, 3), dtype=np.uint64).astype(np.uint32).view(np.float32).copy()
    vs[~np.isfinite(vs)] = f32(1.5)
    vs[rng.random(vs.shape) < 0.3] = f32(0.0)  # zero components (as +0)
    extra = np.array([[0, 0, 0], [2.5, 0, -1e-40], [3e38, -3e38, 1e-45], [-0.0, -0.0, -0.0]], np.float32)
    vs = np.concatenate([vs, extra]) + f32(0.0)  # anim_transform's final add: never -0
    T = np.tile(np.eye(4, dtype=np.float32).reshape(16), (len(vs), 1))
    T[:, 12:15] = vs
    with np.errstate(over="ignore", under="ignore", invalid="ignore"):
        ref = general_inverse(T)
    assert ref.dtype == np.float32
    got = closed_form(vs)
    assert np.array_equal(ref.view(np.uint32), got.view(np.uint32))
