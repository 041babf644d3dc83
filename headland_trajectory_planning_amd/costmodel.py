"""Algorithmic byte / flop model of one IPM iteration.

B_iter = 8 * [ 2 (nnzJ + nnzH) + 7 (n_var + n_eq + n_ineq) ]   bytes per problem per
iteration: one evaluation sweep writing g, grad f, J, H; one factor sweep reading
them; the iterate / step / multiplier read-modify-write.

nnzJ / nnzH are *structural* counts of the NLP of R/obca_py/optimizer.py (no
data-dependent zero elimination; nnzH = lower triangle, per-stage terms summed
without de-duplicating overlaps -> an upper bound):
  dynamics Jacobian rows  : RK2 (time-opt) 24 entries / interval, Euler 13  (+5 identity)
  dynamics Hessian (lower): RK2 19 / interval, Euler 4       (sympy, tools/gen_dynamics.py)
  objective Hessian       : u-u 3, v-v 1, (v,tau)+(tau,tau) 2 per interval; jerk cross
                            u_{i+1}u_i 4 (+ u_i tau_i 2 + u_{i+1} tau_i 2 when time-opt)
  per (stage, obstacle, body) pair with e_m, e_n edges:
      J: c1 e_m, c2 2 (e_n + e_m + 1), c3 e_n + e_m + 2
      H: lam-lam e_m (e_m + 1)/2, (theta, x, y)-lam 3 e_m, theta-theta 1
"""


def nlp_counts(N, M, K, topt, obs_edges, body_edges):
    P = N * M * K
    n_var = 5 * N + 2 * (N - 1) + N * (sum(body_edges) * M + sum(obs_edges) * K) + (N - 1 if topt else 0) + 5
    n_eq = 5 + 5 * (N - 1) + 5 + 2 * P
    n_ineq = 2 * P
    return n_var, n_eq, n_ineq


def structural_nnz(N, M, K, topt, obs_edges, body_edges):
    jdyn, hdyn = (24, 19) if topt else (13, 4)
    hobj = 3 + 1 + (2 if topt else 0)
    hjerk = 4 + (4 if topt else 0)
    nnzJ = 5 + (N - 1) * (5 + jdyn) + 10
    nnzH = (N - 1) * (hdyn + hobj) + max(0, N - 2) * hjerk + 5
    for em in obs_edges:
        for en in body_edges:
            nnzJ += N * (em + 2 * (en + em + 1) + (en + em + 2))
            nnzH += N * (em * (em + 1) // 2 + 3 * em + 1)
    return nnzJ, nnzH


def bytes_per_iteration(N, M, K, topt, obs_edges, body_edges):
    n_var, n_eq, n_ineq = nlp_counts(N, M, K, topt, obs_edges, body_edges)
    nnzJ, nnzH = structural_nnz(N, M, K, topt, obs_edges, body_edges)
    return 8 * (2 * (nnzJ + nnzH) + 7 * (n_var + n_eq + n_ineq))
