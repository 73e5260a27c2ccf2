"""The library's device-block cache (acmmp_engine.hip DevPool; VERDICT r5 #4,
ADVICE r5): engines of two sizes created and destroyed under the default cap,
a small cap, the cache off (0) and a negative setting (off, not unbounded);
blocks are reused, the cache never exceeds its cap, acmmp_release_device_cache
gives everything back, an out-of-memory hipMalloc releases the cache and
retries, and the maps are bit-identical whatever the cache does.

ACMMP_DEVICE_POOL_MB is read once per process, so each setting runs in a
child process (one at a time: a single GPU user alive at any moment)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import hashlib, json, sys
sys.path.insert(0, sys.argv[1])
import numpy as np
import torch
from acmmp_amd import ACMMP, default_params, scene
from acmmp_amd.engine import device_cache_bytes, release_device_cache

mode = sys.argv[2]
s1 = scene.make_scene(num_views=5, width=160, height=120)
s2 = scene.make_scene(num_views=5, width=640, height=480)
rec = {"bytes": {}, "hash": {}}

def run(sc, tag):
    cams, imgs = sc.problem(0, 4)
    p = default_params()
    p.max_iterations = 2
    with ACMMP(0) as eng:
        eng.set_params(p)
        eng.set_images(cams, imgs)
        eng.RunPatchMatch()
        rec["bytes"][tag + "_live"] = device_cache_bytes(0)
        h = hashlib.sha256(eng.plane_hypotheses().tobytes() + eng.costs().tobytes()).hexdigest()
    rec["bytes"][tag] = device_cache_bytes(0)
    rec["hash"][tag] = h

if mode == "oom":
    # the large engine's blocks go to the cache; torch then takes every
    # byte it can get, so the small engine's first hipMalloc fails unless
    # the library gives its cached blocks back and retries
    run(s2, "big")
    hold, chunk = [], 256 << 20
    while chunk >= (1 << 20):
        try:
            hold.append(torch.empty(chunk, dtype=torch.uint8, device="cuda"))
        except torch.OutOfMemoryError:
            chunk >>= 1
    rec["held_mib"] = sum(t.numel() for t in hold) >> 20
    rec["free_after_fill"] = torch.cuda.mem_get_info()[0]
    run(s1, "small")
    del hold
else:
    run(s1, "a")
    run(s2, "b")
    run(s1, "a2")
    release_device_cache(0)
    rec["bytes"]["released"] = device_cache_bytes(0)
    run(s1, "a3")
    release_device_cache(-1)
    rec["bytes"]["released_all"] = device_cache_bytes(-1)
print("RESULT " + json.dumps(rec))
"""


def _child(pool_mb, mode="seq"):
    env = dict(os.environ)
    if pool_mb is None:
        env.pop("ACMMP_DEVICE_POOL_MB", None)
    else:
        env["ACMMP_DEVICE_POOL_MB"] = str(pool_mb)
    r = subprocess.run([sys.executable, "-c", CHILD, ROOT, mode], env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("RESULT ")][-1]
    return json.loads(line[len("RESULT "):])


@pytest.fixture(scope="module")
def runs():
    return {k: _child(v) for k, v in (("default", None), ("cap1", 1), ("off", 0), ("negative", -5))}


def test_maps_identical_with_cache_on_and_off(runs):
    ref = runs["off"]["hash"]
    assert ref["a"] == ref["a2"] == ref["a3"]
    for name, r in runs.items():
        assert r["hash"] == ref, name


def test_default_cache_reuses_and_releases(runs):
    b = runs["default"]["bytes"]
    assert b["a"] > 0  # the first engine's blocks were kept
    assert b["b"] > b["a"]  # the second size's blocks joined them
    # the same size again takes its blocks back out of the cache while alive
    assert b["a2_live"] == b["b"] - b["a"], b
    assert b["a2"] == b["b"]
    assert b["released"] == 0 and b["released_all"] == 0, b


def test_small_cap_bounds_the_cache(runs):
    b = runs["cap1"]["bytes"]
    assert max(b.values()) <= 1 << 20, b


def test_zero_and_negative_setting_mean_off(runs):
    for name in ("off", "negative"):
        assert max(runs[name]["bytes"].values()) == 0, (name, runs[name]["bytes"])


def test_out_of_memory_releases_cache_and_retries():
    r = _child(None, "oom")
    b = r["bytes"]
    assert b["big"] > 0, b  # blocks were cached before the fill
    assert b["small_live"] < b["big"], (r, "the small engine's allocation did not go through the release path")
    ref = _child(0)["hash"]["a"]
    assert r["hash"]["small"] == ref
