"""The multi-GPU gather's deadline logic (csrc/comm_wait.hpp) on the CPU: the waits behind the
non-blocking RCCL communicator (vcrt_comm_init, the gather in vcrt_draw_next_frame) return
done, failed or timed out -- never block -- so that a lost peer makes DrawNextFrame return
VK_ERROR_DEVICE_LOST instead of hanging rank 0 (reference convention: errors bubble up as
VkResult, VulkanComputeRayTracing.cpp:20-35). Built with g++ from the product header."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def driver(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("commwait") / "comm_wait_driver")
    subprocess.run(["g++", "-O2", "-std=c++17", "-Wall", "-Wextra", "-Werror",
                    "-I", os.path.join(ROOT, "vulkancomputeraytracing_amd", "csrc"),
                    os.path.join(ROOT, "tests", "comm_wait_driver.cpp"), "-o", exe], check=True)
    return exe


def run(exe, **env):
    e = dict(os.environ)
    e.pop("VCRT_COMM_TIMEOUT_MS", None)
    e.update(env)
    out = subprocess.run([exe], capture_output=True, text=True, check=True, env=e).stdout
    return {l.split()[0]: l.split()[1:] for l in out.strip().splitlines()}


def test_wait_outcomes(driver):
    r = run(driver)
    assert r["done_after_5"] == ["done", "5"]
    assert r["failed_after_3"] == ["failed", "3"]
    # the deadline passes at the 50th poll of the 1-ms fake clock, not before
    assert r["pending_forever"][:2] == ["timeout", "50"]
    assert r["done_at_deadline"] == ["done", "50"]
    res, polls, ms = r["real_clock"]
    assert res == "timeout" and 200 <= int(ms) < 1500 and int(polls) > 64
    assert r["default_ms"] == ["120000"]


def test_gather_deadline_scales_with_frame_time(driver):
    """the gather's deadline covers the peers' renders, so a frame slower than the
    base deadline must not be reported as a lost peer; a peer that never sends still times out."""
    r = run(driver)
    assert r["slow_peer"] == ["done", "150", "171"]
    assert r["lost_peer"] == ["timeout", "171"]
    assert r["gather_ms"] == ["120001", str(120000 + int(4 * 2670.5 + 1))]


def test_timeout_from_environment(driver):
    assert run(driver, VCRT_COMM_TIMEOUT_MS="2500")["default_ms"] == ["2500"]
    assert run(driver, VCRT_COMM_TIMEOUT_MS="0")["default_ms"] == ["120000"]
    assert run(driver, VCRT_COMM_TIMEOUT_MS="junk")["default_ms"] == ["120000"]
