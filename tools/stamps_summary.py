import json, sys, numpy as np
for f in sys.argv[1:]:
    d = json.load(open(f)); t = d['per_tile'][1]
    g = np.array(t['gemm_per_layer_per_wave']); e = np.array(t['post_gemm_per_layer_per_wave'])
    print(f, 'tile', t['tile_cycles'], 'hidden gemm', int(np.median(g[1:12].max(1))), 'epi', int(np.median(e.max(1))), 'out', g[12].max(),
          'layer5 first group', t.get('layer5_first_group'))
