"""Host facts of a GPU box that shape the thread budget: CPUs visible, affinity, cgroup CPU quota, memory."""
import json
import os


def _read(path):
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


info = {'cpu_count': os.cpu_count(), 'affinity': len(os.sched_getaffinity(0)),
        'cgroup_cpu_max': _read('/sys/fs/cgroup/cpu.max'), 'cgroup_cpuset': _read('/sys/fs/cgroup/cpuset.cpus.effective'),
        'omp_num_threads': os.environ.get('OMP_NUM_THREADS'), 'loadavg': _read('/proc/loadavg'),
        'mem_total_kb': next((ln.split()[1] for ln in (_read('/proc/meminfo') or '').splitlines()
                              if ln.startswith('MemTotal')), None),
        'cpu_model': next((ln.split(':', 1)[1].strip() for ln in (_read('/proc/cpuinfo') or '').splitlines()
                           if ln.startswith('model name')), None)}
print(json.dumps(info))
