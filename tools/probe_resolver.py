"""Name-resolution timings on a box (the r4h distributed-test hang): the lookups that
torch.distributed's TCPStore (reverse lookup of each peer address, socket.cpp) and gloo's default
device (host name -> address) make, then a 4-rank gloo world on the CPU with and without
GLOO_SOCKET_IFNAME=lo. Prints one JSON line. No GPU."""
import json
import os
import socket
import sys
import time

import torch.multiprocessing as mp


def _t(f):
    t = time.time()
    try:
        r = repr(f())
    except Exception as e:  # noqa: BLE001
        r = "error: " + repr(e)
    return {"s": round(time.time() - t, 3), "r": r[:80]}


def _rank(r, world, port, ifname, q):
    import datetime

    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(r), WORLD_SIZE=str(world))
    if ifname:
        os.environ["GLOO_SOCKET_IFNAME"] = ifname
    t = time.time()
    dist.init_process_group("gloo", rank=r, world_size=world, timeout=datetime.timedelta(seconds=120))
    t1 = time.time()
    g = [dist.new_group([0, 1]), dist.new_group([2, 3]), dist.new_group([0, 2]), dist.new_group([1, 3])]
    t2 = time.time()
    dist.barrier()
    dist.destroy_process_group()
    q.put((r, round(t1 - t, 3), round(t2 - t1, 3), len(g)))


def _world(ifname):
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_rank, args=(r, 4, port, ifname, q)) for r in range(4)]
    t = time.time()
    for p in ps:
        p.start()
    for p in ps:
        p.join(300)
    out = sorted(q.get() for _ in range(4) if not q.empty())
    return {"wall_s": round(time.time() - t, 3), "ranks": out}


if __name__ == "__main__":
    host = socket.gethostname()
    res = {
        "hostname": host,
        "getnameinfo_127": _t(lambda: socket.getnameinfo(("127.0.0.1", 0), socket.NI_NUMERICSERV)),
        "getnameinfo_v4mapped": _t(lambda: socket.getnameinfo(("::ffff:127.0.0.1", 0, 0, 0), socket.NI_NUMERICSERV)),
        "gethostbyname_host": _t(lambda: socket.gethostbyname(host)),
        "getaddrinfo_host": _t(lambda: socket.getaddrinfo(host, None)[:1]),
        "lo_exists": os.path.exists("/sys/class/net/lo"),
    }
    for name, ifn in (("gloo_default", ""), ("gloo_lo", "lo")):
        if len(sys.argv) > 1 and name not in sys.argv[1:]:
            continue
        res[name] = _world(ifn)
    print(json.dumps(res))
