! abi_case_driver.f90 — a Fortran host that analyses one variable through the C ABI.
!
! Used by tests/test_fortran_host.py: Python writes a case file (stream, little-endian):
!   k nx ny nz ix_lim iy_lim wf ntypes (i4) norain (r4) vp (raw cwbl_var_params bytes)
!   x(nx,ny) y(nx,ny) alt(nx,ny,nz) var(nx,ny,nz,k) (r4)
!   per type: family type_id nvar nobs (i4), xyz(3,n) (r4),
!             gts: obs(nvar,n) error(nvar,n) hdxb(nvar,n,k) (r4) qc(nvar,n,k) (i4)
!             radar: obs(n) hdxb(n,k) (r4)
! and this program writes var(nx,ny,nz,k) after cwbl_analyze_var.
program abi_case_driver
    use iso_c_binding
    use letkf_core_gpu
    implicit none
    type gts_in
        real(c_float),  allocatable :: xyz(:,:), obs(:,:), error(:,:), hdxb(:,:,:)
        integer(c_int), allocatable :: qc(:,:,:)
    end type gts_in
    type rad_in
        real(c_float),  allocatable :: xyz(:,:), obs(:), hdxb(:,:)
    end type rad_in
    character(len=512) :: fin, fout
    integer(c_int) :: k, nx, ny, nz, ix_lim, iy_lim, wf, ntypes, fam, tid, nvar, nobs
    real(c_float)  :: norain
    type(cwbl_var_params)                 :: vp
    type(cwbl_init_params)                :: ip
    type(cwbl_slab)                       :: slab
    type(cwbl_stats)                      :: st
    type(cwbl_obs_set)                    :: os
    type(cwbl_gts_obs),   target          :: g(29)
    type(cwbl_radar_obs), target          :: r(4)
    type(gts_in),         target          :: gd(29)
    type(rad_in),         target          :: rd(4)
    real(c_float), allocatable, target    :: x(:,:), y(:,:), alt(:,:,:), var(:,:,:,:)
    integer :: it, ng, nr

    call get_command_argument(1, fin)
    call get_command_argument(2, fout)
    open(10, file=trim(fin), access='stream', form='unformatted', status='old')
    read(10) k, nx, ny, nz, ix_lim, iy_lim, wf, ntypes
    read(10) norain
    read(10) vp
    allocate(x(nx,ny), y(nx,ny), alt(nx,ny,nz), var(nx,ny,nz,0:k-1))
    read(10) x, y, alt, var
    ng = 0
    nr = 0
    do it = 1, ntypes
        read(10) fam, tid, nvar, nobs
        if (fam == 0) then
            ng = ng + 1
            allocate(gd(ng)%xyz(3,nobs), gd(ng)%obs(nvar,nobs), gd(ng)%error(nvar,nobs), &
                     gd(ng)%hdxb(nvar,nobs,0:k-1), gd(ng)%qc(nvar,nobs,0:k-1))
            read(10) gd(ng)%xyz, gd(ng)%obs, gd(ng)%error, gd(ng)%hdxb, gd(ng)%qc
            g(ng) = cwbl_gts_obs(tid, nvar, nobs, 0, c_loc(gd(ng)%xyz), c_loc(gd(ng)%obs), &
                                 c_loc(gd(ng)%error), c_loc(gd(ng)%hdxb), c_loc(gd(ng)%qc))
        else
            nr = nr + 1
            allocate(rd(nr)%xyz(3,nobs), rd(nr)%obs(nobs), rd(nr)%hdxb(nobs,0:k-1))
            read(10) rd(nr)%xyz, rd(nr)%obs, rd(nr)%hdxb
            r(nr) = cwbl_radar_obs(tid, nobs, c_loc(rd(nr)%xyz), c_loc(rd(nr)%obs), &
                                   c_loc(rd(nr)%hdxb))
        end if
    end do
    close(10)

    if (cwbl_abi_version() /= 2) stop "ABI version mismatch"
    ip = cwbl_init_params(k, 0, wf, norain, CWBL_Q1_REPLICATE, 0, 0_c_size_t)
    call cwbl_check(cwbl_init(ip), 'cwbl_init')
    os = cwbl_obs_set(ng, nr, c_loc(g), c_loc(r), CWBL_MEM_HOST, 0)
    call cwbl_check(cwbl_set_obs(os), 'cwbl_set_obs')
    slab = cwbl_slab(nx, ny, nz, nx, ny, ix_lim, iy_lim, CWBL_MEM_HOST, c_loc(x), c_loc(y), &
                     c_loc(alt), c_loc(var))
    call cwbl_check(cwbl_analyze_var(vp, slab, st), 'cwbl_analyze_var')
    print '(a,i0,a,i0,a,i0)', 'fortran host: solved=', st%solved, ' max_p=', st%max_p, &
          ' max_sweeps=', st%max_sweeps
    call cwbl_check(cwbl_finalize(), 'cwbl_finalize')
    open(11, file=trim(fout), access='stream', form='unformatted', status='replace')
    write(11) var
    close(11)
end program abi_case_driver
