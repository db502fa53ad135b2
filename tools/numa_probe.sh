export TMPDIR=/tmp
echo "nodes: $(ls /sys/devices/system/node | grep node | tr '\n' ' ')"
for n in /sys/devices/system/node/node*; do echo "$n cpus $(cat $n/cpulist)"; done
for d in /sys/class/drm/card*/device; do [ -f $d/numa_node ] && echo "$d numa $(cat $d/numa_node) $(cat $d/vendor 2>/dev/null)"; done
python3 -c "import os; a=sorted(os.sched_getaffinity(0)); print('affinity', len(a), a[:8], a[-4:])"
