"""Physical constants (cgs) — CODATA 2018 as used by astropy 4.3.1, the reference's
unit backend, plus the hot-Jupiter planet of ``Planet.from_hot_jupiter`` (core.py:92-106)
evaluated once with astropy (IAU 2015 nominal Jupiter, 0.03 AU orbit, R_sun)."""

H = 6.62607015e-27             # erg s
C = 29979245800.0              # cm s^-1
K_B = 1.380649e-16             # erg K^-1
M_P = 1.67262192369e-24        # g
AMU = 1.6605390666e-24         # g
SIGMA_SB = 5.6703744191844314e-05  # erg cm^-2 s^-1 K^-4 (astropy's derived value)
BAR = 1e6                      # dyn cm^-2 per bar
UM = 1e-4                      # cm per micron

# Planet.from_hot_jupiter(): g = G M_J / R_J^2, m_bar = 2.4 m_p, a/R* = 0.03 AU / R_sun
G_JUPITER = 2478.6519476149147        # cm s^-2
M_BAR_HOT_JUPITER = 4.0142926168559996e-24  # g (== 2.4 * M_P)
A_RSTAR_HOT_JUPITER = 6.450964670116429
M_BAR_DEFAULT = 2.4 * M_P

FLUX_UNIT = "erg / (s cm3)"
