#!/bin/bash
# A/B of ticket-ordered tiles (Launch::ticket, forced by DFMI_DIAG=1
# DFMI_TICKET=1) against blockIdx-ordered tiles on the main bench lines,
# alternating twice on the same box.
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do for t in 0 1; do
  DFMI_DIAG=1 DFMI_TICKET=$t timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --sweep 0.5,0.01 --no-cpu \
      --extra c4,c3 --gather 0 > gpurun_out/tk_$t.json 2> gpurun_out/tk_$t.err || { tail gpurun_out/tk_$t.err; exit 1; }
  python3 - $t $rep <<'PY' | tee -a gpurun_out/ticket_ab.log
import json, sys
t, rep = sys.argv[1], sys.argv[2]
d = json.load(open("gpurun_out/tk_%s.json" % t))
e = d["extra"]
print("rep %s ticket=%s  C2 s=0.5 %.4f ms  s=0.01 %.4f ms  C4 %.4f ms  C3 eq %.4f lt %.4f ms" % (
    rep, t, d["roofline"]["kernel_ms"], d["sweep"]["0.01"]["kernel_ms"] if "0.01" in d.get("sweep", {}) else float("nan"),
    e["c4"]["kernel_ms"], e["c3"]["eq"]["roofline"]["kernel_ms"], e["c3"]["lt"]["roofline"]["kernel_ms"]))
PY
done; done
