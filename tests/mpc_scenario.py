"""Receding-horizon test scenarios (test helper): the caller side of HKDProblem::update
(HKDProblem.cpp:117-222) for a batch sharing one gait clock — which contact the reference gait
has at the moving horizon end, the phase bookkeeping that follows from it, and the inputs
(contacts, x0, references) of each shifted layout.

Gait timeline: phase q of the cycle covers absolute knots [q N, (q + 1) N); every element of the
batch switches contact at the same knots (its own cycle), so the layout stays batch-uniform."""
import numpy as np

from hsddp import synthetic as syn


class Scenario:
    def __init__(self, gaits, n_phases, knots):
        self.gaits, self.N = list(gaits), knots
        self.B = len(self.gaits)
        self.horizons = [knots] * n_phases
        self.reach_end = [0] * n_phases
        self.phase_contacts = [[self.gait_at(b, i * knots) for i in range(n_phases)] for b in range(self.B)]
        self.t0 = 0

    def gait_at(self, b, tau):
        cyc = syn.GAITS[self.gaits[b]]
        return tuple(cyc[(tau // self.N) % len(cyc)])

    @property
    def Kc(self):
        return sum(self.horizons)

    def step(self, n):
        """n simulation steps; returns the contact_change flag of each step (shared by the batch)."""
        flags = []
        for _ in range(n):
            kc = self.Kc                  # invariant over a step: one knot leaves, one arrives
            self.t0 += 1
            end = self.t0 + kc            # the new horizon end (QuadReference::step)
            if self.horizons[0] <= 1:
                self.horizons.pop(0); self.reach_end.pop(0)
                for pc in self.phase_contacts:
                    pc.pop(0)
            else:
                self.horizons[0] -= 1
            new = [self.gait_at(b, end) for b in range(self.B)]
            ch = [new[b] != self.phase_contacts[b][-1] for b in range(self.B)]
            assert all(c == ch[0] for c in ch), "the batch must share its contact-change times"
            cc = int(ch[0])
            if cc and self.reach_end[-1]:
                self.horizons.append(1); self.reach_end.append(0)
                for b in range(self.B):
                    self.phase_contacts[b].append(new[b])
            else:
                self.horizons[-1] += 1
                if cc:
                    self.reach_end[-1] = 1
            flags.append(cc)
        return flags

    def inputs(self, x0):
        """contacts [B][P+1][4] (row P: the contact after the horizon when the last phase has
        reached its end, else its own contact — no touchdown), x0, per-element references."""
        P = len(self.horizons)
        S = sum(n + 1 for n in self.horizons)
        end = self.t0 + self.Kc
        contacts = np.zeros((self.B, P + 1, 4), np.int32)
        rx, ru, rf = np.zeros((self.B, S, 24)), np.zeros((self.B, S, 24)), np.zeros((self.B, S, 12))
        for b in range(self.B):
            pc = list(self.phase_contacts[b])
            pc.append(self.gait_at(b, end + 1) if self.reach_end[-1] else pc[-1])
            contacts[b] = np.array(pc, np.int32)
            rx[b], ru[b], rf[b] = syn._reference_slots(pc, self.horizons, syn.DT, self.t0)
        return {"contacts": contacts, "x0": np.ascontiguousarray(x0), "ref_x": rx, "ref_u": ru, "ref_foot": rf}
