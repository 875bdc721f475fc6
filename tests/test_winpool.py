"""The peer-window pool's policy (trpo-robot-control_amd/csrc/trpo_winpool.h), compiled with gcc and run on
the CPU: windows of healthy contexts are parked up to the pool's capacity and handed back by device and
size; a window whose exchange failed is leaked, never parked (a late push from that group could carry a
tag the next group expects -- ADVICE r05); past the capacity a window is freed only under the HIP runtime
the library was built against, and leaked with ONE warning otherwise (no silent hipFree)."""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(os.path.dirname(HERE), "trpo-robot-control_amd", "csrc")

PROG = r"""
#include <stdio.h>
#include "trpo_winpool.h"
#define CHECK(c) do { if (!(c)) { printf("FAIL line %d: %s\n", __LINE__, #c); return 1; } } while (0)
int main(void) {
    winpool w = {0};
    int warn, buf[64];
    /* a failed exchange's window: leaked, the pool untouched */
    CHECK(winpool_give(&w, &buf[0], 100, 0, 1, 1, &warn) == WINPOOL_LEAKED_FAILED && !warn && w.n == 0);
    /* healthy windows park up to the capacity */
    for (int i = 0; i < WINPOOL_CAP; ++i) CHECK(winpool_give(&w, &buf[i], 100 + (i & 1), i & 2, 0, 0, &warn) == WINPOOL_PARKED && !warn);
    CHECK(w.n == WINPOOL_CAP);
    /* full: freed under the built runtime, leaked with one warning under another */
    CHECK(winpool_give(&w, &buf[40], 100, 0, 0, 1, &warn) == WINPOOL_FREED && !warn);
    CHECK(winpool_give(&w, &buf[41], 100, 0, 0, 0, &warn) == WINPOOL_LEAKED_FULL && warn);
    CHECK(winpool_give(&w, &buf[42], 100, 0, 0, 0, &warn) == WINPOOL_LEAKED_FULL && !warn);   /* warned once */
    CHECK(w.n == WINPOOL_CAP);
    /* take: by device and size, each window once */
    CHECK(winpool_take(&w, 7, 100) == NULL);
    CHECK(winpool_take(&w, 0, 999) == NULL);
    void *p = winpool_take(&w, 2, 101);
    CHECK(p == &buf[3] || p == &buf[7] || p == &buf[11] || p == &buf[15]);
    CHECK(w.n == WINPOOL_CAP - 1);
    int got = 1;
    while (winpool_take(&w, 2, 101)) ++got;
    CHECK(got == 4 && w.n == WINPOOL_CAP - 4);
    /* room again: a healthy window parks */
    CHECK(winpool_give(&w, &buf[50], 100, 0, 0, 0, &warn) == WINPOOL_PARKED);
    puts("ok");
    return 0;
}
"""


def test_winpool_policy(tmp_path):
    src = tmp_path / "winpool_test.c"
    src.write_text(PROG)
    exe = tmp_path / "winpool_test"
    subprocess.run(["gcc", "-std=gnu99", "-Wall", "-Werror", "-fsanitize=address,undefined", "-I", CSRC, str(src),
                    "-o", str(exe)], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True)
    assert r.returncode == 0 and r.stdout.strip() == "ok", r.stdout + r.stderr
