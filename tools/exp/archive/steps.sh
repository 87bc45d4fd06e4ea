# Run GPU steps in order (each a shell command line); a step that FAILS its checks (exit 1, e.g. a red
# test) does not stop the chain, but a time limit (124 / 137), an abort (134) or a crash (139) does:
# after those nothing more touches the GPU in this call.
#   bash tools/exp/steps.sh 'GPU_TAG=x bash tools/gpu.sh tests' 'bash tools/exp/r04_table.sh t'
worst=0
for cmd in "$@"; do
  echo "=== $cmd"
  bash -c "$cmd"; rc=$?
  echo "=== rc=$rc"
  case $rc in
    0) ;;
    1|2) worst=1 ;;
    *) echo "stopping after rc=$rc"; exit $rc ;;
  esac
done
exit $worst
