A="python3 tools/atari_kernel_ab.py"
# (the DQN_C1_CO flag and its kernel were removed after the measurement -- rejected)
for r in 1 2; do
  echo "== old"; TSRL_LIB_PATH=variants/libtsrl_c1old.so timeout -k 10 120 $A > /tmp/o.txt 2>&1 || exit $?; grep conv /tmp/o.txt
  echo "== co"; timeout -k 10 120 $A > /tmp/o.txt 2>&1 || exit $?; grep conv /tmp/o.txt
done
