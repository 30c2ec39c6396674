#!/bin/bash
# Offline ISA of the hiprtc-specialised scan for a pattern set (for reading
# the inner loop): [ISA_HITS=true] [ISA_DEFS=-D..] tools/jit_isa.sh OUTDIR "nt::CtPat<6,8,8,1,4,4,4>" ["tvr list"]
set -eu
out=$1; pats=$2; tvrs=${3:-}
here=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$out"
cat > "$out/j.hip" <<EOT
#include <hip/hip_runtime.h>
#include "nt_scan.h"
using JitSet = nt::CtSet<nt::CtList<$pats>, nt::CtList<$tvrs>>;
#ifdef NT_SCAN_WAVES_EU
#define NT_SCAN_ATTR __attribute__((amdgpu_waves_per_eu(NT_SCAN_WAVES_EU)))
#else
#define NT_SCAN_ATTR
#endif
extern "C" __global__ void __launch_bounds__(256) NT_SCAN_ATTR
nt_scan_jit_lds(const NtProgram* __restrict__ prog, const uint32_t* __restrict__ thr, NtBatch B,
                NtOut O, uint64_t* __restrict__ tmask, unsigned long long* __restrict__ queue,
                uint32_t len_lo, uint32_t len_hi, uint32_t claim, uint32_t nstatic, uint32_t wave_words,
                uint32_t* __restrict__ gscr) {
  extern __shared__ uint32_t smem[];
  nt::scan_reads<JitSet, true, ${ISA_HITS:-false}>(prog, thr, B, O, tmask, queue, len_lo, len_hi, claim, nstatic,
                               smem + (threadIdx.x >> 6) * wave_words);
}
EOT
cd "$out"
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -DNT_ISA_MARKS ${ISA_DEFS:-} -I"$here/telomere-analyzer_amd/csrc" \
  -c --save-temps -Rpass-analysis=kernel-resource-usage j.hip -o j.o 2>&1 | grep -E "VGPRs:|SGPRs:|Occupancy" | sed 's/.*remark: //'
python3 - <<'EOT'
s=open('j-hip-amdgcn-amd-amdhsa-gfx950.s').read()
i=s.index('nt_scan_jit_lds:'); j=s.index('.Lfunc_end',i)
open('k.s','w').write(s[i:j])
EOT
# instruction mix between the chunk markers (both the edge and the interior instances)
python3 - <<'EOT'
import re
s=open('k.s').read().split('\n')
marks=[i for i,l in enumerate(s) if 'NT_CHUNK_BEGIN' in l or 'NT_CHUNK_END' in l]
pairs=[(marks[i],marks[i+1]) for i in range(0,len(marks)-1,2)]
for a,b in pairs:
    body=[l.strip() for l in s[a:b] if l.strip() and not l.strip().startswith(';') and not l.strip().startswith('.')]
    v=sum(1 for l in body if l.startswith('v_')); sa=sum(1 for l in body if l.startswith('s_') and not l.startswith('s_nop')); ds=sum(1 for l in body if l.startswith('ds_'))
    print(f"chunk region lines {a}-{b}: VALU {v} SALU {sa} LDS {ds} (static, all paths)")
EOT
