#!/usr/bin/env bash
# Compatibility entry point: same name, verbs and flags as the reference's
# kind-gpu-sim.sh, implemented by the kgs Python package (MI355X-native).
#   ./kind-gpu-sim.sh {create [rocm]|delete|load|status|bench} [--registry-port=N] [--cluster-name=S] [--image-name=S]
set -euo pipefail
here="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
export PYTHONPATH="${here}${PYTHONPATH:+:${PYTHONPATH}}"
exec "${PYTHON:-python3}" -m kgs "$@"
