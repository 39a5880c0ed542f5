"""The programs' user modules (programs/*/m_user.f90) the driver can run:
the procedure pointers of m_user_methods they set, as Python hooks.

Each hook takes cell centres r (n, 3) in metres (af_r_cc) and returns
values per cell; Simulation calls them per box, ghost cells included."""
import numpy as np


class Sprite3D:
    """programs/3d_sprite/m_user.f90 (BASELINE config 5, sprite_3d.cfg)."""

    e_decay_height = 2.86e3   # m_user.f90:17 (Wait-Spies model)
    scale_height = 7.2e3      # :19
    n_e0 = 1e4                # :20

    @classmethod
    def gas_density(cls, r):
        """gas_density (m_user.f90:34-40): 2.5e25 exp(-z / H)."""
        return 2.5e25 * np.exp(-r[:, 2] / cls.scale_height)

    @classmethod
    def initial_conditions(cls, sim, r):
        """my_init_cond (m_user.f90:42-78): an exponential electron and ion
        profile above 60 km plus the cfg's seeds (electrons for charge type
        <= 0, ions for >= 0); returns (n_e, n_+)."""
        from .driver import density_line
        ne = cls.n_e0 * np.exp((r[:, 2] - 60e3) / cls.e_decay_height)
        ni = ne.copy()
        for sd in sim.seeds:
            dens = density_line(r, sd["r0"], sd["r1"], sd["n0"], sd["n1"], sd["width"],
                                sd["falloff"])
            if sd["type"] <= 0:
                ne = ne + dens
            if sd["type"] >= 0:
                ni = ni + dens
        return ne, ni


USERS = {"s5": Sprite3D}
