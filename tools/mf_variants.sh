# rocprofv3 kernel stats of a probe script (PROBE, default tools/mf_probe.py), one
# run per variant library (build/var/libdcp_<name>.so from tools/variant_probe.sh).
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/mfvar
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
# a spec is VAR or NAME=VAR:ENV1,ENV2 (runtime environment of the probe)
for spec in ${VARS}; do
  v=${spec%%:*}; name=${v%%=*}; v=${v#*=}
  envs=""; [ "$spec" != "${spec#*:}" ] && envs=${spec#*:}
  rm -rf /tmp/pv
  env ${envs//,/ } VAR=$v R=${R:-5} timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pv -o run \
    -- python3 $GRAFT_REPO_ROOT/${PROBE:-tools/mf_probe.py} > $OUT/$name.log 2>&1 || exit $?
  find /tmp/pv -name "*kernel_stats.csv" -exec cp {} $OUT/$name.csv \;
done
python3 - <<'PY'
import csv, glob, os, re
out = os.environ["GRAFT_REPO_ROOT"] + "/gpurun_out/mfvar"
for f in sorted(glob.glob(out + "/*.csv")):
    rows = {r["Name"]: r for r in csv.DictReader(open(f))}
    sel = {re.search(r"k_\w+(<[^>]*>)?", k.split("::")[-1]).group(0): float(r["AverageNs"]) / 1e3
           for k, r in rows.items()
           if any(x in k for x in ("k_mf_pencil<", "k_mf_gather<", "k_mf_fused<", "k_bt_tasks<",
                                   "k_nse_rhs_halfwave", "k_con_gather"))}
    print(os.path.basename(f)[:-4], {k: round(v, 1) for k, v in sel.items()})
PY
