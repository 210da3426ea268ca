import cProfile, pstats, sys, os, io, time
sys.argv=['bench_pool.py']
os.environ['N']='20000'; os.environ['N_CPU']='10'
sys.path.insert(0,'tools'); sys.path.insert(0,'.')
src=open('tools/bench_pool.py').read()
# run only the gpu part under the profiler
src=src.replace('out = {"metric"', 'pr = cProfile.Profile(); pr.enable(); _g = run("gpu_batched", clients, reqs); pr.disable(); s = io.StringIO(); pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(25); print(s.getvalue()); print(_g); sys.exit(0)\nout = {"metric"')
exec(compile(src,'bench_pool','exec'))
