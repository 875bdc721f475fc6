"""The product's text-file parsers (csrc/trpo_textio.c, host side of the file-based entry points) on
well-formed, short, truncated, empty, garbage and non-file inputs -- CPU only.

Semantics are the reference's fscanf("%lf") loops (src/TRPO_FVP.c:670-699 model, :731-762 data): missing
values stay zero, a non-number stops the parse, Std is the last row's.  The same tests run against
the AddressSanitizer + UBSan build of the unit (TRPO_TEXTIO_LIB, tests/test_asan.py).
"""
import ctypes as C
import os

import numpy as np
import pytest

import cases
import oracle
import trpo_amd

_dp = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")


def _lib():
    L = C.CDLL(os.environ.get("TRPO_TEXTIO_LIB") or trpo_amd.LIB_PATH)
    L.trpo_text_load_model.restype = C.c_int
    L.trpo_text_load_model.argtypes = [C.c_char_p, C.c_size_t, _dp]
    L.trpo_text_load_data.restype = C.c_int
    L.trpo_text_load_data.argtypes = [C.c_char_p, C.c_size_t, C.c_size_t, C.c_size_t, _dp, _dp, C.c_void_p,
                                      C.c_void_p, C.c_void_p]
    L.trpo_text_parse_doubles.restype = C.c_size_t
    L.trpo_text_parse_doubles.argtypes = [C.c_char_p, _dp, C.c_size_t]
    return L


L = _lib()
O, A = 15, 3
ROW = 3 * A + O + 1


def model(path, P):
    th = np.full(P, np.nan)
    rc = L.trpo_text_load_model(str(path).encode(), P, th)
    return rc, th


def data(path, n, std0=None):
    obs = np.full(n * O, np.nan)
    std = np.array(std0 if std0 is not None else [np.nan] * A, dtype=np.float64)
    mean, act, adv = np.full(n * A, np.nan), np.full(n * A, np.nan), np.full(n, np.nan)
    rc = L.trpo_text_load_data(str(path).encode(), O, A, n, obs, std, mean.ctypes.data, act.ctypes.data,
                               adv.ctypes.data)
    return rc, obs.reshape(n, O), std, mean.reshape(n, A), act.reshape(n, A), adv


def test_fixture_files_match_the_oracle_reader():
    """The reference's own ArmTestModel.txt / ArmTestData.txt parse to what the oracle's reader gives."""
    layers = [15, 16, 16, 3]
    P = 582
    rc, th = model(os.path.join(cases.GOLDEN, "ArmTestModel.txt"), P)
    assert rc == 0
    np.testing.assert_array_equal(th, oracle.load_model(os.path.join(cases.GOLDEN, "ArmTestModel.txt"), layers))
    rc, obs, std, mean, act, adv = data(os.path.join(cases.GOLDEN, "ArmTestData.txt"), 3150)
    assert rc == 0
    ob2, st2 = oracle.load_data(os.path.join(cases.GOLDEN, "ArmTestData.txt"), layers, 3150)
    np.testing.assert_array_equal(obs, ob2)
    np.testing.assert_array_equal(std, st2)


def test_missing_file_and_directory(tmp_path, capfd):
    assert model(tmp_path / "nope.txt", 10)[0] == -1
    assert "[ERROR] Cannot open Model File" in capfd.readouterr().err
    assert data(tmp_path / "nope.txt", 2)[0] == -1
    assert "[ERROR] Cannot open Data File" in capfd.readouterr().err
    assert model(tmp_path, 10)[0] == -1                 # a directory is not a text file
    assert data(tmp_path, 2)[0] == -1


@pytest.mark.parametrize("text,expect", [
    ("", []),
    ("\n\n  \t\r\n", []),
    ("1 2 3", [1, 2, 3]),
    ("1\n2\n3", [1, 2, 3]),                           # no trailing newline
    ("1.5e-3\n-2\n", [1.5e-3, -2]),
    ("1 2 abc 4", [1, 2]),                            # a non-number stops the parse (fscanf)
    ("1 2 3 4 5 6 7 8 9 10 11 12", list(range(1, 11))),  # more than asked for: the first P
    ("nan inf -inf", [np.nan, np.inf, -np.inf]),
    ("1e999 -1e999 1e-999", [np.inf, -np.inf, 0.0]),
    ("0x10 1", [16, 1]),                              # strtod == %lf: hex floats too
    ("3.", [3.0]),
])
def test_model_short_garbage(tmp_path, text, expect):
    f = tmp_path / "m.txt"
    f.write_text(text)
    rc, th = model(f, 10)
    assert rc == 0
    want = np.zeros(10)
    want[:len(expect)] = expect
    np.testing.assert_array_equal(th, want)


def test_model_binary_garbage(tmp_path):
    rng = np.random.default_rng(5)
    for k in range(20):
        f = tmp_path / ("g%d" % k)
        f.write_bytes(rng.integers(0, 256, size=int(rng.integers(0, 4096)), dtype=np.uint8).tobytes())
        rc, th = model(f, 64)
        assert rc == 0 and th.shape == (64,) and not np.isnan(th).all()


def _row(i):
    return [0.1 * i, 0.2, 0.3,          # Mean
            1.0 + i, 2.0 + i, 3.0 + i,  # Std
            *[i + 0.01 * j for j in range(O)], 7.0, 8.0, 9.0, -1.0 * i]


def test_data_full_and_last_std(tmp_path):
    rows = [_row(i) for i in range(5)]
    f = tmp_path / "d.txt"
    f.write_text("\n".join(" ".join("%.17g" % v for v in r) for r in rows) + "\n")
    rc, obs, std, mean, act, adv = data(f, 4)                # the first N rows only
    assert rc == 0
    for i in range(4):
        np.testing.assert_array_equal(obs[i], rows[i][6:6 + O])
        np.testing.assert_array_equal(mean[i], rows[i][:3])
        np.testing.assert_array_equal(act[i], rows[i][6 + O:9 + O])
        assert adv[i] == rows[i][-1]
    np.testing.assert_array_equal(std, rows[3][3:6])          # Std of the LAST parsed row


@pytest.mark.parametrize("cut", [0, 1, 4, 10, ROW - 1, ROW + 5])
def test_data_truncated(tmp_path, cut):
    """A file that ends inside row 2: the missing values are zero and Std keeps the last value read."""
    vals = _row(0) + _row(1) + _row(2)[:cut]
    f = tmp_path / "d.txt"
    f.write_text(" ".join("%.17g" % v for v in vals))
    rc, obs, std, mean, act, adv = data(f, 4)
    assert rc == 0
    full = np.zeros((4, ROW))
    flat = np.array(vals)
    full.flat[:len(flat)] = flat
    stds = [np.array(_row(0)[3:6]), np.array(_row(1)[3:6])]
    for i in range(2, 4):                                     # Std of a short row: previous values
        prev = stds[-1]
        got_std = full[i, 3:6].copy()
        nread = max(0, min(ROW, len(flat) - i * ROW))
        for j in range(3):
            if 3 + j >= nread:
                got_std[j] = prev[j]
        stds.append(got_std)
    for i in range(4):
        np.testing.assert_array_equal(obs[i], full[i, 6:6 + O])
        assert adv[i] == full[i, -1]
    np.testing.assert_array_equal(std, stds[-1])


def test_data_garbage_midway(tmp_path):
    f = tmp_path / "d.txt"
    f.write_text(" ".join("%.17g" % v for v in _row(0)) + "\n1 2 3 junk 5\n" + " ".join("1" for _ in range(ROW)))
    rc, obs, std, mean, act, adv = data(f, 3)
    assert rc == 0
    np.testing.assert_array_equal(obs[0], _row(0)[6:6 + O])
    assert not obs[1:].any() and not adv[1:].any()            # fscanf never passes the bad token
    np.testing.assert_array_equal(std, _row(0)[3:6])           # row 1 stopped after its Mean: row 0's Std


def test_data_empty_and_zero_rows(tmp_path):
    f = tmp_path / "d.txt"
    f.write_text("")
    rc, obs, std, mean, act, adv = data(f, 3, std0=[0.5, 0.5, 0.5])
    assert rc == 0 and not obs.any()
    np.testing.assert_array_equal(std, [0.5, 0.5, 0.5])
    rc = data(f, 0, std0=[0.5, 0.5, 0.5])[0]
    assert rc == 0
