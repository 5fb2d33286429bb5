import os, sys, faulthandler, time
sys.path[:0] = ['/root/repo', '/root/repo/scaled-mmd-gan_amd', '/root/repo/tests']
os.environ.setdefault('GRAFT_REPO_ROOT', '.')
import torch, torch.multiprocessing as mp
import test_gpu_dist as T

def worker(rank, world, port, q):
    faulthandler.dump_traceback_later(40, exit=True)
    print('rank', rank, 'start', flush=True)
    try:
        T._worker(rank, world, port, q)
    except Exception as e:
        import traceback; traceback.print_exc()
        q.put(('err', rank, repr(e)))
        raise
    print('rank', rank, 'done', flush=True)

if __name__ == '__main__':
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = T._free_port()
    ps = [ctx.Process(target=worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps: p.start()
    for _ in range(2):
        print(q.get(timeout=90)[:3], flush=True)
    for p in ps: p.join(60); print('exit', p.exitcode, flush=True)
