"""HOCON parser, typed params (reference validations/defaults) and the native data parser."""
import glob
import os

import numpy as np
import pytest

from ytk_learn_amd.config.hocon import ConfigError, parse, parse_file
from ytk_learn_amd.config.params import CommonParams, LineSearchParams, gbdt_params_from_config
from ytk_learn_amd.ops._ext import native
from ytk_learn_amd.utils.errors import YtkLearnError

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"


def test_hocon_syntax():
    c = parse('''
    # comment
    a : 1, b = "x" // trailing
    c { d : [1, 2, 3,], e.f : true }
    c.g = 1E-8
    c { h : ??? }
    arr : [{k : 1}, {k : 2}]
    s : ${c.d}
    u : gradient_boosting
    ''')
    assert c.get_int("a") == 1 and c.get_string("b") == "x"
    assert c.get_list("c.d") == [1, 2, 3]
    assert c.get_bool("c.e.f") is True
    assert c.get_double("c.g") == 1e-8
    assert c.get("c.h") == "???"
    with pytest.raises(ConfigError):
        c.get_string("c.h")  # placeholder must be set
    assert c.get_list("arr")[1]["k"] == 2
    assert c.get_list("s") == [1, 2, 3]
    assert c.get_string("u") == "gradient_boosting"
    assert c.with_value("c.d", [9]).get_list("c.d") == [9]
    assert c.get_list("c.d") == [1, 2, 3]  # immutable


def test_repo_configs_parse_and_validate():
    for f in glob.glob(os.path.join(ROOT, "config", "model", "*.conf")):
        c = parse_file(f).with_overrides({"data.train.data_path": "x", "model.data_path": "m",
                                          "data.max_feature_dim": 10, "model.field_dict_path": "f"})
        if f.endswith("gbdt.conf"):
            gp, dp, mp = gbdt_params_from_config(c)
            assert gp.tree.max_leaf_cnt == 32  # min(128, 2^5): GBDTOptimizationParams.java:148-154
        else:
            p = CommonParams.from_config(c)
            assert p.line_search.mode == "wolfe"


@pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "config")), reason="reference configs not available")
def test_reference_configs_parse():
    files = glob.glob(os.path.join(REF, "config/model/*.conf")) + glob.glob(os.path.join(REF, "demo/**/*.conf"),
                                                                              recursive=True)
    assert len(files) >= 9
    for f in files:
        parse_file(f)


def test_param_validations():
    c = parse_file(os.path.join(ROOT, "config", "model", "linear.conf")).with_overrides(
        {"data.train.data_path": "x", "model.data_path": "m"})
    with pytest.raises(YtkLearnError):
        LineSearchParams.from_config(c.with_value("optimization.line_search.backtracking.c1", 2.0))
    with pytest.raises(YtkLearnError):
        CommonParams.from_config(c.with_value("data.delim.y_delim", "###"))
    with pytest.raises(YtkLearnError):
        CommonParams.from_config(c.with_value("data.y_sampling", ["0.5"]))
    g = parse_file(os.path.join(ROOT, "config", "model", "gbdt.conf")).with_overrides(
        {"data.train.data_path": "x", "model.data_path": "m", "data.max_feature_dim": 3})
    with pytest.raises(YtkLearnError):
        gbdt_params_from_config(g.with_value("optimization.uniform_base_prediction", 1.5))
    gp, _, _ = gbdt_params_from_config(g.with_value("type", "random_forest"))
    assert gp.tree.learning_rate == 1.0  # RF forces lr = 1


def _parse(text, **opts):
    return native().parse_buffer(text.encode(), opts)


def test_parser_basic_and_errors():
    r = _parse("2###1###a:1,b:2,a:3###0.7\n\n1###0###c:1.5f\nbad line\n1###1,0###\n", max_error_tol=1)
    assert r["n_rows"] == 3 and r["n_errors"] == 1
    np.testing.assert_array_equal(r["weight"], [2, 1, 1])
    assert r["names"] == ["a", "b", "c"]
    np.testing.assert_array_equal(r["val"], [3, 2, 1.5])  # repeated name keeps the last value
    np.testing.assert_array_equal(r["label_ptr"], [0, 1, 2, 4])
    np.testing.assert_array_equal(r["init"], np.float32([0.7]))
    np.testing.assert_array_equal(r["row_line"], [0, 2, 4])
    with pytest.raises(RuntimeError):
        _parse("bad\nworse\n", max_error_tol=1)


def test_parser_hash_matches_guava_vector():
    # MurmurHash3_x64_128("hello", seed 0): h1 = 0xcbd8a7b341bd9b02 (Guava asLong)
    assert native().murmur3_128_aslong("hello", 0) & (2 ** 64 - 1) == 0xcbd8a7b341bd9b02
    r = _parse("1###0###a:1,b:2\n", feature_hash=True, hash_bucket=7, hash_seed=39916801)
    assert all(n.startswith("hash_") and int(n[5:]) < 7 for n in r["names"])


def test_parser_sharding_and_sampling():
    lines = "".join(f"1###{i % 2}###f{i}:1\n" for i in range(100))
    a = _parse(lines, line_mod=3, line_rem=1)
    assert a["n_rows"] == 33 and a["row_line"][0] == 1
    s = _parse(lines, y_sampling=[0.5, 1.0], sample_seed=3)
    kept0 = (s["labels"] == 0).sum()
    assert 10 <= kept0 <= 40 and (s["labels"] == 1).sum() == 50
    assert np.all(s["weight"][s["labels"] == 0] == 2.0)  # weight *= 1 / rate


def test_parser_multithreaded_deterministic():
    g = np.random.default_rng(0)
    lines = "".join("1###%d###%s\n" % (i % 2, ",".join(f"x{j}:{g.random():.3f}" for j in g.integers(0, 500, 8)))
                    for i in range(60000))
    for opts in ({}, {"y_sampling": [0.3, 1.0], "sample_seed": 5}):
        a = _parse(lines, threads=1, **opts)
        b = _parse(lines, threads=8, **opts)
        assert a["names"] == b["names"] and a["n_rows"] == b["n_rows"]
        for k in ("indptr", "feat", "val", "weight", "labels", "row_line"):
            np.testing.assert_array_equal(a[k], b[k])


def test_parser_java_float_grammar():
    r = _parse("1###1###a:NaN,b:1.5f,c:2d,d:+3\n1###1###a:nan\n1###1###a:inf\n1###1###a:Infinity\n"
               "1###1###a:1e400\n", max_error_tol=10)
    assert r["n_rows"] == 1 and r["n_errors"] == 4  # lowercase nan/inf and +-Infinity rejected
    assert np.isnan(r["val"][0]) and list(r["val"][1:]) == [1.5, 2.0, 3.0]


def test_java_random_stream():
    n = native()
    # java.util.Random(42): nextDouble 0.7275636800328681, nextGaussian 1.1419053154730547
    assert abs(n.java_random(42, 1, 3)[0] - 0.7275636800328681) < 1e-16
    assert abs(n.java_random(42, 1, 0, 0.0, 1.0)[0] - 1.1419053154730547) < 1e-15
    assert abs(n.java_random(0, 1, 2)[0] - 0.73096776) < 1e-7


def _nearest_f32(s):
    """Correctly rounded float32 of a decimal string (exact rational arithmetic, ties to even)."""
    from fractions import Fraction
    x = Fraction(s)
    f = np.float32(float(s))
    best = None
    for c in (np.nextafter(f, np.float32(-np.inf)), f, np.nextafter(f, np.float32(np.inf))):
        if not np.isfinite(c):
            continue
        d = abs(Fraction(float(c)) - x)
        key = (d, int(np.frombuffer(np.float32(c).tobytes(), np.uint32)[0]) & 1)
        if best is None or key < best[0]:
            best = (key, c)
    return best[1]


def test_parser_float_fast_path_correctly_rounded():
    """The parser's fast decimal path (mantissa < 2^24, |exp10| <= 10) and the from_chars
    fallback both give the correctly rounded float32 (Java Float.parseFloat semantics)."""
    rng = np.random.default_rng(3)
    toks = ["0", "-0", "5.", ".5", "1e3", "1E-3", "-2.5e+2", "16777215", "16777217", "0.1", "3.4e38",
            "1.17549435e-38", "123456789", "1234567890", "0.000001234", "9.99999e9", "7e10", "7e11", "1e-10",
            "1e-11", "+4.25", "2.5f", "-0.0000"]
    for _ in range(400):
        m = int(rng.integers(0, 10 ** int(rng.integers(1, 10))))
        e = int(rng.integers(-14, 14))
        toks.append(f"{'-' if rng.random() < 0.3 else ''}{m}e{e}")
        toks.append(f"{rng.normal() * 10.0 ** int(rng.integers(-6, 8)):.{int(rng.integers(1, 10))}g}")
    line = "1###0###" + ",".join(f"f{i}:{t}" for i, t in enumerate(toks))
    r = _parse(line + "\n")
    assert r["n_errors"] == 0
    got = np.asarray(r["val"], np.float32)
    for t, g in zip(toks, got):
        want = _nearest_f32(t.rstrip("fF").lstrip("+"))
        assert np.float32(g).tobytes() == np.float32(want).tobytes() or (g == 0 and want == 0), (t, g, want)
    for bad in ["-", ".", "-.", "1e", "e5", "1.2.3", "nan", "inf", "--1"]:
        rb = _parse(f"1###0###a:{bad}\n", max_error_tol=1)
        assert rb["n_errors"] == 1, bad
