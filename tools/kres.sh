#!/bin/bash
# Device-only compile of one kernel file with hipcc's resource-usage remarks (VGPR / SGPR / spills /
# LDS / occupancy per kernel) and the gfx950 assembly: tools/kres.sh csrc/kernels/X.hip [defines...]
# -> /tmp/kres/X.res.txt, /tmp/kres/X.s
set -eo pipefail
f=$(readlink -f "${1:?kernel file}"); shift
mkdir -p /tmp/kres
n=$(basename "$f" .hip)
TI=$(python -c "import torch,os;print(os.path.dirname(torch.__file__)+'/include')")
R=$(cd "$(dirname "$0")/.." && pwd)
flags="-std=c++17 -O3 --offload-arch=gfx950 --cuda-device-only -D__HIP_PLATFORM_AMD__=1 -DUSE_ROCM=1 -DTORCH_API_INCLUDE_EXTENSION_H -DTORCH_EXTENSION_NAME=_C -I$R/csrc/include -I$TI -I$TI/torch/csrc/api/include -I/usr/include/python3.10 $*"
hipcc $flags -Rpass-analysis=kernel-resource-usage -c "$f" -o /tmp/kres/$n.o 2> /tmp/kres/$n.res.txt || { grep error /tmp/kres/$n.res.txt | head; exit 1; }
hipcc $flags -S "$f" -o /tmp/kres/$n.s 2>/dev/null
grep -E "Function Name|VGPRs:|AGPRs|Scratch|Spill|Occupancy|LDS Size" /tmp/kres/$n.res.txt | sed -e 's/.*remark: *//' -e 's/ \[-Rpass.*//'
