"""Exactness of the multiply-high division by the clock periods (config.h
Div64 / fdiv): both engines divide femtosecond stamps with it, so it must
equal true integer division for every 64-bit dividend."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SRC = r'''
#include "model/config.h"
#include <cstdio>
#include <random>
using namespace asim;
int main() {
  std::mt19937_64 g(12345);
  const uint64_t ds[] = {1, 2, 3, 5, 7, 10, 641, 691085, 883392, 1176471, 1000000, 714286, 999999937ull,
                         (1ull << 32) - 1, (1ull << 32) + 1, 0x8000000000000001ull, 0xffffffffffffffffull,
                         1ull << 40, 6700417};
  uint64_t bad = 0, n = 0;
  auto chk = [&](uint64_t x, const Div64& v, uint64_t d) { ++n; if (fdiv(x, v) != x / d) ++bad; };
  for (uint64_t d : ds) {
    const Div64 v = make_div64(d);
    for (int i = 0; i < 200000; ++i) {
      const uint64_t x = g() >> (g() % 64);
      chk(x, v, d);
    }
    for (uint64_t k = 0; k < 2000; ++k) {  // around multiples of d and the top of the range
      const uint64_t m = d * k;
      chk(m, v, d); chk(m + 1, v, d); if (m) chk(m - 1, v, d);
      chk(~0ull - k, v, d);
    }
  }
  for (int i = 0; i < 2000; ++i) {  // random divisors
    const uint64_t d = (g() >> (g() % 63)) | 1;
    const Div64 v = make_div64(d);
    for (int j = 0; j < 200; ++j) chk(g() >> (g() % 64), v, d);
  }
  printf("%llu %llu\n", (unsigned long long)bad, (unsigned long long)n);
  return bad != 0;
}
'''


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_fdiv_equals_integer_division(tmp_path):
    src = tmp_path / "fd.cc"
    src.write_text(SRC)
    exe = tmp_path / "fd"
    subprocess.check_call(["g++", "-std=c++17", "-O2", "-I", os.path.join(ROOT, "csrc"), str(src), "-o", str(exe)])
    out = subprocess.run([str(exe)], capture_output=True, text=True)
    bad, n = map(int, out.stdout.split())
    assert out.returncode == 0 and bad == 0 and n > 4_000_000, out.stdout
