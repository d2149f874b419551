"""Output format (image/ppm.rs): the product writer vs the reference KATs and,
byte for byte, vs the oracle's writer."""
import numpy as np


def test_ppm_reference_kats(rt):
    c = rt.Canvas(5, 3)  # ppm.rs:90-109
    c.set_pixel(0, 0, rt.Color(1.5, 0.0, 0.0))
    c.set_pixel(2, 1, rt.Color(0.0, 0.5, 0.0))
    c.set_pixel(4, 2, rt.Color(-0.5, 0.0, 1.0))
    assert c.to_ppm() == (b"P3\n5 3\n255\n"
                          b"255 0 0 0 0 0 0 0 0 0 0 0 0 0 0\n"
                          b"0 0 0 0 0 0 0 128 0 0 0 0 0 0 0\n"
                          b"0 0 0 0 0 0 0 0 0 0 0 0 0 0 255\n")
    c = rt.Canvas(10, 2)  # ppm.rs:127-150
    for j in range(2):
        for i in range(10):
            c.set_pixel(i, j, rt.Color(1.0, 0.8, 0.6))
    line1 = b"255 204 153 255 204 153 255 204 153 255 204 153 255 204 153 255 204\n"
    line2 = b"153 255 204 153 255 204 153 255 204 153 255 204 153\n"
    assert c.to_ppm() == b"P3\n10 2\n255\n" + (line1 + line2) * 2


def test_quantizer_rules(rt):
    # ppm.rs:111-118 plus Rust `round()` / saturating `as u8` edge cases
    v = np.array([0.0, 255.0, -0.5, 1.5, 0.5, 0.1, np.nan, np.inf, -np.inf, -0.0,
                  0.5 / 255, (0.5 - 1e-12) / 255, 254.5 / 255])
    assert rt.quantize_u8(v).tolist() == [0, 255, 0, 255, 128, 26, 0, 255, 0, 0, 1, 0, 255]


def test_ppm_bytes_match_oracle(rt, oracle):
    rng = np.random.default_rng(7)
    for (h, w) in [(1, 1), (3, 5), (7, 23), (40, 31), (2, 70), (1, 0), (0, 3)]:
        img = rng.uniform(-0.2, 1.3, size=(h, w, 3))
        if img.size:
            img.flat[::17] = 0.1  # exact .5 ties after scaling
            img.flat[::29] = np.nan
        assert rt.canvas_to_ppm(img) == oracle.canvas_to_ppm(img)


def test_ppm_row_parallel_writer_matches_oracle(rt, oracle):
    """Canvases large enough for the row-parallel host writer (threads over
    row ranges; every token's position computed before the breaks are walked)."""
    rng = np.random.default_rng(11)
    vals = np.array([0.0, 1 / 255, 9 / 255, 10 / 255, 99 / 255, 100 / 255, 1.0, 0.5 / 255, np.nan, -1.0, 2.0])
    for (h, w) in [(300, 301), (97, 1024), (1000, 71)]:
        img = rng.choice(vals, size=(h, w, 3))
        img[::3] = rng.uniform(-0.2, 1.3, size=img[::3].shape)
        assert rt.canvas_to_ppm(img) == oracle.canvas_to_ppm(img)


def test_ppm_rounding_edges_and_widths_match_oracle(rt, oracle):
    """The table-driven writer (libm-free rounding, 4-byte token stores):
    every quarter step of every quantisation level, the exact .5 boundaries
    and their neighbours, NaN / inf / huge, and widths 1..37 (every line-break
    position and the last token of a row) against the oracle."""
    rng = np.random.default_rng(5)
    for w in range(1, 38):
        a = rng.uniform(-0.1, 1.1, (3, w, 3))
        vals = [0.5 / 255, np.nextafter(0.5 / 255, 0), np.nan, 254.5 / 255, np.nextafter(254.5 / 255, 0), np.inf,
                -np.inf, 1e300, 0.0, -0.0, 2.5 / 255, 3.5 / 255] + list(np.arange(1024) / 4 / 255)
        k = (w * 7) % len(vals)
        flat = a.reshape(-1)
        n = min(flat.size, len(vals))
        flat[:n] = (vals[k:] + vals[:k])[:n]
        ref = oracle.canvas_to_ppm(a)
        ref = ref.encode() if isinstance(ref, str) else ref
        assert rt.canvas_to_ppm(a) == ref, w
    big = rng.uniform(0, 1, (9, 500, 3))  # rows long enough for many breaks, and the threaded path
    ref = oracle.canvas_to_ppm(big)
    assert rt.canvas_to_ppm(big) == (ref.encode() if isinstance(ref, str) else ref)
