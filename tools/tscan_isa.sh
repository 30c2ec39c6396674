#!/bin/bash
# Offline ISA of the bundle scan (nt_tscan.h) for a pattern set, as the hiprtc
# build would make it: tools/tscan_isa.sh OUTDIR "nt::CtPat<6,8,8,1,4,4,4>" ["tvr list"] [L]
set -eu
out=$1; pats=$2; tvrs=${3:-}; L=${4:-100}
here=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$out"
cat > "$out/t.hip" <<EOT
#include <hip/hip_runtime.h>
#include "nt_tscan.h"
using PatL = nt::CtList<$pats>;
using TvrL = nt::CtList<$tvrs>;
using JitT = nt::TProg<PatL, TvrL, $L>;
constexpr int kTsW = nt::ts_lds_words<JitT::kNP, JitT::kL>();
constexpr int kTsNW = 40960 / kTsW < 4 ? 40960 / kTsW : 4;
extern "C" __global__ void __launch_bounds__(kTsNW * 64) __attribute__((amdgpu_waves_per_eu(1)))
nt_tscan_jit(NtBatch B, NtOut O, uint64_t* __restrict__ tmask,
             unsigned long long* __restrict__ queue, uint32_t thr_full) {
  __shared__ uint32_t tsl[kTsNW * kTsW];
  nt::tscan_bundles<JitT, PatL, TvrL>(B, O, tmask, queue, thr_full, tsl + (threadIdx.x >> 6) * kTsW);
}
EOT
cd "$out"
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off ${ISA_DEFS:-} -I"$here/telomere-analyzer_amd/csrc" \
  -c --save-temps -Rpass-analysis=kernel-resource-usage t.hip -o t.o 2>&1 | grep -E "error|VGPRs:|AGPRs:|SGPRs:|Spill|Occupancy|ScratchSize" | sed 's/.*remark: //'
python3 - <<'EOT'
import collections
s=open('t-hip-amdgcn-amd-amdhsa-gfx950.s').read()
i=s.index('nt_tscan_jit:'); j=s.index('.Lfunc_end',i)
k=s[i:j]; open('k.s','w').write(k)
c=collections.Counter(l.split()[0] for l in k.split('\n') if l.strip() and l.strip()[0] in 'vsdbg' and not l.strip().startswith(';'))
tot=sum(v for kk,v in c.items() if kk.startswith('v_'))
print('static VALU', tot, 'SALU', sum(v for kk,v in c.items() if kk.startswith('s_')))
print(sorted(((kk,v) for kk,v in c.items() if kk.startswith('v_')), key=lambda x:-x[1])[:30])
EOT
