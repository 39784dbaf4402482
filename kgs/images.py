"""Build the in-tree images (replaces the reference's clone + sed-patch + build of
upstream Go plugins, kind-gpu-sim.sh:144-228 -- here everything is built from
this repository, so there is nothing to clone, pin or patch; Q6/Q8 vanish).

* ``images/Dockerfile.deviceplugin`` -> ``localhost:<port>/amdgpu-dp:dev``
* ``images/Dockerfile.rocm-test``    -> ``localhost:<port>/kgs-rocm-test:dev``
  (PyTorch-ROCm base; gfx950 kernels compiled at image build). On a CPU-only
  host the same Dockerfile is built on a slim Python base and the entrypoint
  prints the reference's fake-GPU greeting.
"""
from __future__ import annotations

from . import config as C
from .cluster import REPO_ROOT


AMDSMI_LIB_REPO = "kgs-amdsmi-lib"
AMDSMI_LIB_TAG = "7.0"


def build_images(p, workload: bool = True, plugin: bool = True, amdsmi_lib: bool = False) -> int:
    rt = p.ensure_runtime()
    p.start_registry()
    if amdsmi_lib:
        # the light source of the plugin's amd-smi stage (images/Dockerfile.amdsmi-lib)
        tag = f"{p.s.registry_host}/{AMDSMI_LIB_REPO}:{AMDSMI_LIB_TAG}"
        rt.cr("build", "-t", tag, "--build-arg", f"UBUNTU_IMAGE={p.s.library_image('ubuntu:22.04')}",
              "-f", str(REPO_ROOT / "images" / "Dockerfile.amdsmi-lib"), str(REPO_ROOT))
        if rt.name == "docker":
            rt.cr("push", tag)
        print(f"amd-smi stage image: {tag}  (use: --rocm-dev-image={tag})")
    if plugin:
        tag = f"{p.s.registry_host}/{C.PLUGIN_IMAGE_REPO}:{C.PLUGIN_IMAGE_TAG}"
        rt.cr("build", "-t", tag, *p.s.plugin_build_args(),
              "-f", str(REPO_ROOT / "images" / "Dockerfile.deviceplugin"), str(REPO_ROOT))
        if rt.name == "docker":
            rt.cr("push", tag)
    if workload:
        if p.topology is None and p.s.fake_gpus is None:
            p.discover()
        base = p.s.library_image(C.PY_SLIM_IMAGE) if p.fake else p.s.rocm_image(p.s.rocm_base_image)
        tag = f"{p.s.registry_host}/{C.WORKLOAD_IMAGE_REPO}:{C.WORKLOAD_IMAGE_TAG}"
        rt.cr("build", "-t", tag, "--build-arg", f"BASE_IMAGE={base}",
              "--build-arg", f"BUILD_NATIVE={'0' if p.fake else '1'}",
              "-f", str(REPO_ROOT / "images" / "Dockerfile.rocm-test"), str(REPO_ROOT))
        if rt.name == "docker":
            rt.cr("push", tag)
    return 0
