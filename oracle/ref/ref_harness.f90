! ref_harness.f90 — drives the reference's own compiled code to produce golden vectors.
!
! TEST INFRASTRUCTURE ONLY (built by oracle/ref/build_ref.sh into oracle/_ref/).
! Real reference code exercised: module param / config (read_namelist) / eigen
! (set_optimal_workspace_for_eigen, inverse_matrix, sqrt_matrix) / kdtree2_module
! (kdtree2_create, kdtree2_r_nearest) / localization (build_tree, get_lz, destroy_tree,
! Gaspari_Cohn_1999) and the source text of letkf_yoyb, letkf_solve and letkf_tune_q (see
! build_ref.sh).  Only letkf_driver's point loop (module_letkf_core.f90:209-240) is written
! out here (ref_driver.inc); letkf_driver itself needs the MPI decomposition.
!
! Usage: ref_harness <mode> <in.bin> <out.bin>,
! modes: consts | solve | search | gc | driver | tuneq | ingest
! (ingest also compiles module_projection and the source text of the obs readers
! read_gts_omboma / read_alt_info / get_alt / read_radar; see build_ref.sh)
! All files are unformatted stream (little-endian int32 / real32 / real64).
module harness_lib
    use param
    use config
    use eigen
    use kdtree2_module
    use ref_extract
    use projection, only : proj_type
    use ref_ingest
    use localization, only : lz_structure, build_tree, get_lz, destroy_tree, Gaspari_Cohn_1999
    implicit none

    character(len=512) :: fin, fout

contains

    ! read_namelist (module_config.f90:328-397) with nmember = k (plus any extra namelist
    ! lines per group), then the set-up calls of cwb_letkf.f90:37-38.
    subroutine setup_k(k, ctl, obsl, infl)
        integer, intent(in)                    :: k
        character(len=*), intent(in), optional :: ctl, obsl, infl
        character(len=600)  :: nmlfile
        nmlfile = trim(fout)//'.nml'
        open(31, file=trim(nmlfile), status='replace', action='write')
        write(31, '(a)') '&control'
        write(31, '(a,i0)') ' nmember = ', k
        if (present(ctl)) write(31, '(a)') ctl
        write(31, '(a)') '/'
        write(31, '(a)') '&projection'
        write(31, '(a)') '/'
        write(31, '(a)') '&observations'
        if (present(obsl)) write(31, '(a)') obsl
        write(31, '(a)') '/'
        write(31, '(a)') '&inflation'
        if (present(infl)) write(31, '(a)') infl
        write(31, '(a)') '/'
        close(31)
        call read_namelist(trim(nmlfile))
        open(31, file=trim(nmlfile), status='old')
        close(31, status='delete')
        call set_optimal_workspace_for_eigen(nmember)
        call set_ensemble_constants(nmember)
    end subroutine setup_k

    subroutine do_consts
        real, parameter :: r2 = gc1999 * gc1999          ! module_localization.f90:202
        call setup_k(8)
        open(21, file=trim(fout), access='stream', form='unformatted', status='replace')
        write(21) gc1999, r2, nmember_inv, nmember_1_inv
        close(21)
    end subroutine do_consts

    ! letkf_solve KATs.  in: k npts use_rtpp use_rtps (i4) multi_infl rtpp_a rtps_a (r4),
    ! then per point p (i4) xb(k) yo(p) yb(k,p) (r4).  out: per point xa(k) (r4), lam(k) (r8)
    subroutine do_solve
        integer :: k, npts, irtpp, irtps, ip, p, info
        real    :: multi_infl, rtpp_a, rtps_a, inflat
        real,   allocatable :: xb(:), yo(:), yb(:,:), xa(:)
        real*8, allocatable :: amat(:,:), yb8(:,:), lam(:)
        integer :: i
        open(40, file=trim(fin), access='stream', form='unformatted', status='old')
        read(40) k, npts, irtpp, irtps
        read(40) multi_infl, rtpp_a, rtps_a
        call setup_k(k)
        inflat = (nmember-1) / multi_infl                    ! module_letkf_core.f90:68
        open(21, file=trim(fout), access='stream', form='unformatted', status='replace')
        allocate(xb(k), xa(k), amat(k,k), lam(k))
        do ip = 1, npts
            read(40) p
            allocate(yo(p), yb(k,p), yb8(k,p))
            read(40) xb, yo, yb
            ! eigenvalues as inverse_matrix obtains them (module_eigen.f90:48-49) from the
            ! matrix letkf_solve forms (module_letkf_core.f90:628-649)
            yb8 = dble(yb)
            amat = 0d0
            do i = 1, k
                amat(i,i) = 1d0
            end do
            call dsyrk('l', 'n', k, p, 1d0, yb8, k, dble(inflat), amat, k)
            call dcopy(k*k, amat, 1, evect, 1)
            call dsyevd('v', 'l', k, evect, k, eval, work, lwork, iwork, liwork, info)
            lam = eval
            xa = letkf_solve(xb, yo, yb, inflat, irtpp /= 0, rtpp_a, irtps /= 0, rtps_a)
            write(21) xa, lam
            deallocate(yo, yb, yb8)
        end do
        close(40)
        close(21)
    end subroutine do_solve

    ! get_lz KATs for a single obs type (no Q1 mixing), through the reference's compiled
    ! build_tree / get_lz (module_localization.f90:35-167, 188-331): the points are the vr
    ! radar type (module_radar.f90:13-16), whose namelist entries (radar_nml%vr%use_it,
    ! %max_lz_pts, %hclr(1), %vclr(1)) go through read_namelist.
    ! in: nobs nq max_lz (i4) hclr vclr (r4) xyz(3,nobs) q(3,nq) (r4)
    ! out: per query nfound (i4) idx(max_lz) (i4, 1-based, 0 padded) r2(max_lz) (r4)
    subroutine do_search
        integer :: nobs, nq, max_lz, iq, nlz
        real    :: hclr, vclr
        real, allocatable :: q(:,:)
        type(cwb_radar) :: rad
        type(lz_structure), dimension(:), allocatable :: lz
        integer, allocatable :: idx(:)
        real,    allocatable :: dis(:)
        character(len=400) :: obsl
        logical :: ok, fail
        open(40, file=trim(fin), access='stream', form='unformatted', status='old')
        read(40) nobs, nq, max_lz
        read(40) hclr, vclr
        allocate(rad%radarobs(num_radar_indexes))
        rad%radarobs(vr)%nobs = nobs
        allocate(rad%radarobs(vr)%xyz(3,nobs), q(3,nq), idx(max_lz), dis(max_lz))
        read(40) rad%radarobs(vr)%xyz, q
        close(40)
        write(obsl, '(a,i0,a,es16.8e3,a,es16.8e3)') ' radar_nml%vr%use_it = T'//char(10)// &
            ' radar_nml%vr%max_lz_pts = ', max_lz, char(10)//' radar_nml%vr%hclr(1) = ', hclr, &
            char(10)//' radar_nml%vr%vclr(1) = ', vclr
        call setup_k(8, obsl=trim(obsl))
        ok = build_tree(rad % radarobs, 1)
        if (.not. ok) stop "do_search: build_tree built no tree"
        open(21, file=trim(fout), access='stream', form='unformatted', status='replace')
        do iq = 1, nq
            fail = get_lz('radar', lz, 1, q(:,iq))
            idx = 0
            dis = 0.
            nlz = 0
            if (.not. fail) then
                nlz = size(lz(1) % idx)
                idx(1:nlz) = lz(1) % idx
                dis(1:nlz) = lz(1) % r2
            end if
            write(21) nlz, idx, dis
            if (allocated(lz)) deallocate(lz)
        end do
        close(21)
        call destroy_tree
    end subroutine do_search

    subroutine do_gc
        integer :: n, i
        real, allocatable :: x(:), y(:)
        open(40, file=trim(fin), access='stream', form='unformatted', status='old')
        read(40) n
        allocate(x(n), y(n))
        read(40) x
        close(40)
        do i = 1, n
            y(i) = Gaspari_Cohn_1999(x(i))
        end do
        open(21, file=trim(fout), access='stream', form='unformatted', status='replace')
        write(21) y
        close(21)
    end subroutine do_gc

    ! letkf_tune_q KATs.  in: k nx ny nz (i4), q(nx,ny,nz,k) (r4).  out: q after the call
    subroutine do_tuneq
        integer :: k, nx, ny, nz
        real, allocatable :: q(:,:,:,:)
        open(40, file=trim(fin), access='stream', form='unformatted', status='old')
        read(40) k, nx, ny, nz
        call setup_k(k)
        allocate(q(nx, ny, nz, k))
        read(40) q
        close(40)
        call letkf_tune_q(nz, q)
        open(21, file=trim(fout), access='stream', form='unformatted', status='replace')
        write(21) q
        close(21)
    end subroutine do_tuneq

    ! Obs readers and projection KATs (module_gts_omboma.f90:48-506,704-1049,
    ! module_radar.f90:30-118, module_projection.f90:21-50), run in the directory that holds
    ! the files, as cwb_letkf.f90:46-52 names them: member m (1-based) reads gts_letkf_mmm
    ! with obs_gts, and VR_/MR_/MD_/MK_letkf_mmm; projection_nml at its defaults
    ! (module_config.f90:70-75).  The distribution (gts_distribute / radar_distribute) takes
    ! every array but hdxb / qc from the root reader, member 1 (cwb_letkf.f90:46-57), and
    ! member m's hdxb(:,:,m-1) / qc(:,:,m-1) from member m's reader.
    ! in:  k, n (i4), has(5) (i4: gts, VR, MR, MD, MK), lon(n), lat(n) (r4)
    ! out: xy(2,n) (r4); per GTS type with nobs > 0: type, nvar, nobs (i4), id (5 chars each),
    !      lat, lon, alt (nobs), xyz(3,nobs), obs(nvar,nobs), error(nvar,nobs) (r4), then per
    !      member hdxb(nvar,nobs) (r4), then per member qc(nvar,nobs) (i4); 0 (i4); per radar
    !      type with nobs > 0: type, nobs, obs, lat, lon, alt, xyz(3,nobs), per member
    !      hdxb(nobs); 0
    subroutine do_ingest
        integer :: k, n, has(5), m, t, i
        real, allocatable :: lon(:), lat(:)
        real :: xy(2)
        character(len=3) :: proc
        type(proj_type) :: proj
        type(wrfda_gts), allocatable :: g(:)
        type(cwb_radar), allocatable :: r(:)
        character(len=2), parameter :: rnames(4) = (/ 'MR', 'VR', 'MD', 'MK' /)
        integer, parameter :: rflag(4) = (/ 3, 2, 4, 5 /)    ! dbz, vr, zdr, kdp -> has()
        open(40, file=trim(fin), access='stream', form='unformatted', status='old')
        read(40) k, n
        read(40) has
        allocate(lon(n), lat(n))
        read(40) lon, lat
        close(40)
        call setup_k(k)
        call proj % init()
        open(21, file=trim(fout), access='stream', form='unformatted', status='replace')
        do i = 1, n
            xy = proj % lonlat_to_xy(lon(i), lat(i))
            write(21) xy
        end do
        allocate(g(k), r(k))
        do m = 1, k
            allocate(g(m) % platform(num_gts_indexes), r(m) % radarobs(num_radar_indexes))
            write(proc, '(i3.3)') m
            if (has(1) /= 0) call read_gts_omboma(g(m), proj, 'gts_letkf_'//proc, 'obs_gts')
            do t = 1, num_radar_indexes
                if (has(rflag(t)) /= 0) &
                    call read_radar(r(m), proj, rnames(t)//'_letkf_'//proc, rnames(t))
            end do
        end do
        do t = 1, num_gts_indexes
            associate (p => g(1) % platform(t))
                if (p % nobs <= 0) cycle
                write(21) t, size(p % obs, 1), p % nobs
                write(21) p % id
                write(21) p % lat, p % lon, p % alt, p % xyz, p % obs, p % error
                do m = 1, k
                    write(21) g(m) % platform(t) % hdxb(:, :, m-1)
                end do
                do m = 1, k
                    write(21) g(m) % platform(t) % qc(:, :, m-1)
                end do
            end associate
        end do
        write(21) 0
        do t = 1, num_radar_indexes
            associate (p => r(1) % radarobs(t))
                if (p % nobs <= 0) cycle
                write(21) t, p % nobs
                write(21) p % obs, p % lat, p % lon, p % alt, p % xyz
                do m = 1, k
                    write(21) r(m) % radarobs(t) % hdxb(:, m-1)
                end do
            end associate
        end do
        write(21) 0
        close(21)
    end subroutine do_ingest

    include 'ref_driver.inc'

end module harness_lib

program ref_harness
    use harness_lib
    implicit none
    character(len=512) :: mode

    call get_command_argument(1, mode)
    call get_command_argument(2, fin)
    call get_command_argument(3, fout)

    select case (trim(mode))
    case ('consts')
        call do_consts
    case ('solve')
        call do_solve
    case ('search')
        call do_search
    case ('gc')
        call do_gc
    case ('driver')
        call do_driver
    case ('tuneq')
        call do_tuneq
    case ('ingest')
        call do_ingest
    case default
        stop "ref_harness: unknown mode"
    end select
end program ref_harness
