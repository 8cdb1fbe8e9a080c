# r5e: helper waves poll the hand-off flag and load the sums (h1) vs ring DMA by waves 4-7 only (d1) vs all (d0)
# (logs: profiles/r5e_helper_ab.txt)
