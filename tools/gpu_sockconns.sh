set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for c in 2 4 8; do
  timeout -k 10 300 python3 -u bench.py --sock --sock-conns $c --no-cpu-baseline > gpurun_out/sockconns_$c.json 2> gpurun_out/sockconns_$c.err || { tail -5 gpurun_out/sockconns_$c.err; exit 1; }
  python3 -c "
import json,sys; d=json.load(open('gpurun_out/sockconns_$c.json'))
o=d.get('one_connection') or {}
print($c, d['value'], d['wire_GBps'], d['ceiling_GBps'], d['ceiling_cold_GBps'], d['wire_frac_of_cold_ceiling'], d['verified'], '| one', o.get('value'), o.get('wire_frac_of_cold_ceiling'))"
done
