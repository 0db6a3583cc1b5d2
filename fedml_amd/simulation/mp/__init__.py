"""Message-passing simulation ("MPI" mode of the reference, `simulation/mpi_p2p_mp/*`).

Each rank is an OS process (torchrun + TCP transport) or a thread (LOOPBACK transport). Rank 0
is the server. Every algorithm the reference ships under mpi_p2p_mp is wired here, including the
ones its SimulatorMPI leaves as ``pass`` (Appendix A #6)."""
